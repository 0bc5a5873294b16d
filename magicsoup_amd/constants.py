"""Simulation-wide constants.

Mirrors the reference's ``python/magicsoup/constants.py:1-10`` (codon size, gas constant,
nucleotide alphabet, spec tuple types). The nucleotide *order* ``T, C, G, A`` matters: it fixes the
enumeration order of codon/token tables built by :mod:`magicsoup_amd.models.genetics`.
"""
from itertools import product as _product

CODON_SIZE = 3  # nucleotides per codon
GAS_CONSTANT = 8.31446261815324  # J / (K * mol)

ALL_NTS = ("T", "C", "G", "A")
ALL_CODONS = {a + b + c for a, b, c in _product(ALL_NTS, repeat=3)}

# ((dom_type, i0, i1, i2, i3), dom_start, dom_end)
DomainSpecType = tuple[tuple[int, int, int, int, int], int, int]
# (domains, cds_start, cds_end, is_fwd)
ProteinSpecType = tuple[list[DomainSpecType], int, int, bool]

# numeric guards of the kinetics integrator (reference kinetics.py:9-13)
EPS = 1e-36
MAX = 1e36
MIN = -1e36
