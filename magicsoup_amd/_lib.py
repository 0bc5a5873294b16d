"""The reference's native function surface (``magicsoup._lib``, ``rust/lib.rs:182-202``).

The reference's tests and users call its pyo3 module directly (e.g.
``tests/fast/test_genetics.py:62-93``). These are the same 12 functions with the same argument
lists and return shapes, backed by this package's C++ host core (``magicsoup_amd._host``, OpenMP)
instead of Rust + rayon. ``import magicsoup._lib`` resolves here. World operations do not go
through this surface: on a GPU they run as HIP kernels over device arenas.
"""
from __future__ import annotations

import numpy as np

from magicsoup_amd.ops import native
from magicsoup_amd.utils import util as _util

__all__ = [
    "dist_1d", "free_moores_nghbhd", "point_mutations", "recombinations", "get_coding_regions", "extract_domains",
    "reverse_complement", "translate_genomes", "get_neighbors", "divide_cells_if_possible", "move_cells",
    "get_proteome",
]


# ---------------------------------------------------------------------------- util (rust/util.rs)
def dist_1d(a: int, b: int, m: int) -> int:
    """Circular distance of ``a`` and ``b`` on a line of length ``m`` (``rust/lib.rs:18-21``)."""
    return _util.dist_1d(a, b, m)


def free_moores_nghbhd(x: int, y: int, positions: list[tuple[int, int]], map_size: int) -> list[tuple[int, int]]:
    """Moore neighbours of (x, y) on the torus not in ``positions`` (``rust/lib.rs:23-31``)."""
    return _util.free_moores_nghbhd(x, y, positions, map_size)


# ---------------------------------------------------------------------------- mutations
def point_mutations(seqs: list[str], p: float, p_indel: float, p_del: float) -> list[tuple[str, int]]:
    """``(mutated sequence, index)`` of every changed sequence (``rust/lib.rs:35-44``)."""
    return native.host().point_mutations(list(seqs), float(p), float(p_indel), float(p_del))


def recombinations(seq_pairs: list[tuple[str, str]], p: float) -> list[tuple[str, str, int]]:
    """``(new a, new b, pair index)`` of every recombined pair (``rust/lib.rs:46-53``)."""
    return native.host().recombinations(list(seq_pairs), float(p))


# ---------------------------------------------------------------------------- genetics
def get_coding_regions(seq: str, min_cds_size: int, start_codons: list[str], stop_codons: list[str],
                       is_fwd: bool) -> list[tuple[int, int, bool]]:
    """``(start, stop end, is_fwd)`` of every CDS of one strand (``rust/lib.rs:57-66``)."""
    return native.host().get_coding_regions(seq, int(min_cds_size), list(start_codons), list(stop_codons), bool(is_fwd))


def extract_domains(genome: str, cdss: list[tuple[int, int, bool]], dom_size: int, dom_type_size: int,
                    dom_type_map: dict[str, int], one_codon_map: dict[str, int], two_codon_map: dict[str, int]):
    """Protein specs of the CDSs (``rust/lib.rs:68-87``)."""
    return native.host().extract_domains(genome, [tuple(c) for c in cdss], int(dom_size), int(dom_type_size),
                                         dict(dom_type_map), dict(one_codon_map), dict(two_codon_map))


def reverse_complement(seq: str) -> str:
    """Reverse complement (``rust/lib.rs:89-92``; characters other than TCGA are dropped)."""
    return native.host().reverse_complement(seq)


def translate_genomes(genomes: list[str], start_codons: list[str], stop_codons: list[str], domain_map: dict[str, int],
                      one_codon_map: dict[str, int], two_codon_map: dict[str, int], dom_size: int,
                      dom_type_size: int):
    """Proteome specs of every genome (``rust/lib.rs:94-118``)."""
    tables = native.host().TranslationTables(list(start_codons), list(stop_codons), dict(domain_map),
                                             dict(one_codon_map), dict(two_codon_map), int(dom_size),
                                             int(dom_type_size))
    return tables.translate_genomes(list(genomes))


# ---------------------------------------------------------------------------- world
def _pos_array(positions) -> np.ndarray:
    return np.asarray(positions, dtype=np.int32).reshape(-1, 2)


def get_neighbors(from_idxs: list[int], to_idxs: list[int], positions: list[tuple[int, int]],
                  map_size: int) -> list[tuple[int, int]]:
    """Unique ``(small, large)`` pairs within Chebyshev distance 1 on the torus
    (``rust/lib.rs:122-133``)."""
    pos = _pos_array(positions)
    out = native.host().get_neighbors(np.asarray(from_idxs, dtype=np.int32), np.asarray(to_idxs, dtype=np.int32),
                                      pos, int(map_size), int(map_size), True)
    return [(int(a), int(b)) for a, b in np.asarray(out).reshape(-1, 2)]


def divide_cells_if_possible(cell_idxs: list[int], positions: list[tuple[int, int]], n_cells: int,
                             map_size: int) -> tuple[list[int], list[int], list[tuple[int, int]]]:
    """(dividing cells that found a free Moore neighbour, their children's indices n_cells.., the
    children's positions) in list order (``rust/lib.rs:135-146``)."""
    pos = _pos_array(positions)
    S = int(map_size)
    parents, cpos = native.host().divide_cells(np.asarray(cell_idxs, dtype=np.int32), pos, S, S, 0, S, True, None)
    parents = [int(p) for p in np.asarray(parents)]
    children = list(range(int(n_cells), int(n_cells) + len(parents)))
    return parents, children, [(int(x), int(y)) for x, y in np.asarray(cpos).reshape(-1, 2)]


def move_cells(cell_idxs: list[int], positions: list[tuple[int, int]],
               map_size: int) -> tuple[list[tuple[int, int]], list[int]]:
    """(new positions, moved cells) for cells moving to a free Moore neighbour; the others stay
    as obstacles (``rust/lib.rs:148-156``)."""
    pos = _pos_array(positions)
    S = int(map_size)
    moved, npos = native.host().move_cells(np.asarray(cell_idxs, dtype=np.int32), pos, S, S, 0, S, True, None)
    return [(int(x), int(y)) for x, y in np.asarray(npos).reshape(-1, 2)], [int(c) for c in np.asarray(moved)]


# ---------------------------------------------------------------------------- kinetics
def get_proteome(proteome, vmaxs, kms, hills, signs, reacts, trnspts, effectors, molecules: list[str]) -> list[dict]:
    """Protein dicts (``Protein.from_dict`` format) of one proteome from its per-domain mapped
    values (``rust/lib.rs:160-176``, ``rust/kinetics.rs``): catalytic domains put molecules with a
    negative signed stoichiometry on the left; transporters export when the signed entry is
    negative; a regulatory effector index >= m is transmembrane."""
    m = len(molecules)
    out = []
    for pi, (doms, cds_start, cds_end, is_fwd) in enumerate(proteome):
        dl = []
        for di, (idxs, start, end) in enumerate(doms):
            t = idxs[0]
            spec: dict = {"start": start, "end": end}
            sign = signs[pi][di]
            if t == 1:
                lft, rgt = [], []
                for mi, n in enumerate(reacts[pi][di]):
                    sn = n * sign
                    if sn > 0:
                        rgt.extend([molecules[mi]] * abs(n))
                    elif sn < 0:
                        lft.extend([molecules[mi]] * abs(n))
                spec.update(km=kms[pi][di], vmax=vmaxs[pi][di], reaction=(lft, rgt))
            elif t == 2:
                vec = trnspts[pi][di]
                mi = next(i for i, d in enumerate(vec) if d != 0)
                spec.update(km=kms[pi][di], vmax=vmaxs[pi][di], is_exporter=vec[mi] * sign < 0, molecule=molecules[mi])
            elif t == 3:
                vec = effectors[pi][di]
                i = next(i for i, d in enumerate(vec) if d != 0)
                spec.update(km=kms[pi][di], hill=hills[pi][di], is_transmembrane=i >= m,
                            is_inhibiting=vec[i] * sign < 0, effector=molecules[i % m])
            dl.append({"spec": spec, "type": {1: "C", 2: "T", 3: "R"}.get(t, " ")})
        out.append({"cds_start": cds_start, "cds_end": cds_end, "is_fwd": is_fwd, "domains": dl})
    return out
