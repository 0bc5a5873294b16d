"""Synthetic random chemistries for scaling benchmarks (BASELINE.json configs such as
"16 molecules / 32 reactions" and "64 molecules / 256 reactions").

Molecule names are prefixed (``syn<m>_<i>``) so several synthetic chemistries and the named examples
can coexist in one process.
"""
from __future__ import annotations

import random

from magicsoup_amd.models.containers import Chemistry, Molecule


def make_chemistry(n_molecules: int = 16, n_reactions: int = 32, seed: int = 0, max_side: int = 3) -> Chemistry:
    rng = random.Random(seed)
    mols = [
        Molecule(
            f"syn{n_molecules}_{i}",
            float(rng.randint(10, 400)) * 1e3,
            diffusivity=1.0 if i % 8 == 0 else 0.1,
            permeability=1.0 if i % 8 == 0 else 0.0,
        )
        for i in range(n_molecules)
    ]
    reacts: list[tuple[list[Molecule], list[Molecule]]] = []
    seen = set()
    while len(reacts) < n_reactions:
        k_l, k_r = rng.randint(1, max_side), rng.randint(1, max_side)
        picks = rng.sample(mols, k_l + k_r) if k_l + k_r <= n_molecules else rng.choices(mols, k=k_l + k_r)
        lhs, rhs = sorted(picks[:k_l]), sorted(picks[k_l:])
        key = (tuple(m.name for m in lhs), tuple(m.name for m in rhs))
        if key in seen or (key[1], key[0]) in seen or set(lhs) & set(rhs):
            continue
        seen.add(key)
        reacts.append((lhs, rhs))
    return Chemistry(molecules=mols, reactions=reacts)
