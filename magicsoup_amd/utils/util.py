"""Small sequence / math helpers of the public API.

Behaviour follows the reference ``python/magicsoup/util.py:10-125``: ``round_down``, ``closest_value``,
``randstr``, ``random_genome`` (uniform TCGA with excluded-substring removal and refill), ``variants``
(N/R/Y template expansion), ``codons`` and the torus helpers ``dist_1d`` / ``free_moores_nghbhd``.
The torus helpers are plain Python here (they are O(1) / O(8) per call); the bulk neighbourhood work
of the simulation runs in the native kernels of :mod:`magicsoup_amd.ops`.
"""
from typing import Iterable
from itertools import product
import math
import random
import string

from magicsoup_amd.constants import ALL_NTS, CODON_SIZE

_LABEL_CHARS = string.ascii_uppercase + string.ascii_lowercase + string.digits

# IUPAC-style wildcards understood by `variants`
_WILDCARDS = {"N": ("T", "C", "G", "A"), "R": ("A", "G"), "Y": ("C", "T")}


def round_down(d: float, to: int = 3) -> int:
    """Largest multiple of ``to`` that is <= ``d``."""
    return math.floor(d / to) * to


def closest_value(values: Iterable[float], key: float) -> float:
    """Element of ``values`` (or key of a dict) closest to ``key``; first one wins ties."""
    best = None
    best_d = math.inf
    for v in values:
        dv = abs(v - key)
        if dv < best_d:
            best, best_d = v, dv
    return best  # type: ignore[return-value]


def randstr(n: int = 12) -> str:
    """Random label of ``n`` characters over [A-Za-z0-9] (62 symbols)."""
    return "".join(random.choices(_LABEL_CHARS, k=n))


def _strip(seq: str, excl: list[str]) -> str:
    for pat in excl:
        if pat:
            seq = seq.replace(pat, "")
    return seq


def random_genome(s: int = 500, excl: list[str] | None = None) -> str:
    """Uniformly random nucleotide string of length ``s``.

    Every occurrence of a sequence in ``excl`` is cut out and the genome is refilled with fresh random
    nucleotides until it is ``s`` long again (excluded patterns may still appear on the reverse
    complement, exactly as in the reference).
    """
    out = "".join(random.choices(ALL_NTS, k=s))
    if not excl:
        return out
    out = _strip(out, excl)
    while len(out) != s:
        out = _strip(out + "".join(random.choices(ALL_NTS, k=s - len(out))), excl)
    return out


def variants(seq: str) -> list[str]:
    """All nucleotide strings matching a template with wildcards N (any), R (A/G), Y (C/T)."""
    slots = [_WILDCARDS.get(ch, (ch,)) for ch in seq]
    return ["".join(d) for d in product(*slots)]


def codons(n: int, excl_codons: list[str] | None = None) -> list[str]:
    """All sequences of ``n`` codons, skipping any sequence that contains an excluded codon in frame."""
    seqs = variants("N" * n * CODON_SIZE)
    if not excl_codons:
        return seqs
    excl = set(excl_codons)
    return [
        s
        for s in seqs
        if not any(s[i : i + CODON_SIZE] in excl for i in range(0, n * CODON_SIZE, CODON_SIZE))
    ]


def dist_1d(a: int, b: int, m: int) -> int:
    """Distance between ``a`` and ``b`` on a circular line of length ``m``."""
    d = abs(a - b)
    return min(d, m - d)


def moores_nghbhd(x: int, y: int, map_size: int) -> list[tuple[int, int]]:
    """The 8 toroidal Moore neighbours of (x, y), in the reference order (rust/util.rs:30-46)."""
    m = map_size
    e, w = (x + 1) % m, (x - 1) % m
    s, n = (y + 1) % m, (y - 1) % m
    return [(w, n), (w, y), (w, s), (x, n), (x, s), (e, n), (e, y), (e, s)]


def free_moores_nghbhd(
    x: int, y: int, positions: list[tuple[int, int]], map_size: int
) -> list[tuple[int, int]]:
    """Moore neighbours of (x, y) that are not listed in ``positions``."""
    occ = set(map(tuple, positions))
    return [d for d in moores_nghbhd(x, y, map_size) if d not in occ]
