"""Genome -> proteome translation tables and API.

Table construction follows the reference ``python/magicsoup/genetics.py:58-178``:

* a domain is ``(n_dom_type_codons + 5)`` codons: a type prefix, three 1-codon tokens and one 2-codon
  token (``dom_size`` = 21 nt by default);
* domain-type prefixes are all ``n_dom_type_codons``-codon sequences without a *start* codon, shuffled,
  with ``int(p * n)`` of them assigned to catalytic (1), transporter (2) and regulatory (3) types;
* 1-codon tokens 1..61 enumerate the non-stop codons; 2-codon tokens 1..3904 enumerate the 6-mers
  whose first codon is not a stop.

Translation itself runs in the native core (single-source scan in ``csrc/include/ms_common.h``):
the OpenMP host module for Python lists / CPU worlds and the gfx950 kernel in ``csrc/hip`` for
device-resident genome arenas.
"""
from __future__ import annotations

import random
import warnings

import numpy as np

from magicsoup_amd.constants import CODON_SIZE, ProteinSpecType
from magicsoup_amd.utils.util import codons
from magicsoup_amd.ops import native


def _n_of(p: float, n: int, what: str) -> int:
    k = int(p * n)
    if k == 0 and p > 0.0:
        warnings.warn(
            f"There will be no {what}."
            f" Increase dom_type_size to accomodate low probabilities of having {what}."
        )
    return k


class Genetics:
    """Transcription / translation rules of a world.

    Arguments:
        start_codons: Codons that open a coding sequence (CDS).
        stop_codons: Codons that close a CDS.
        p_catal_dom, p_transp_dom, p_reg_dom: Chance that a random domain-type prefix encodes a
            catalytic, transporter or regulatory domain.
        n_dom_type_codons: Codons in the domain-type prefix.

    A CDS runs from any start codon to the first in-frame stop codon, on the forward strand and on
    the reverse complement. Every CDS with at least one catalytic or transporter domain becomes a
    protein. Assign a custom instance to ``world.genetics`` to change the rules of a world.
    """

    def __init__(
        self,
        start_codons: tuple[str, ...] = ("TTG", "GTG", "ATG"),
        stop_codons: tuple[str, ...] = ("TGA", "TAG", "TAA"),
        p_catal_dom: float = 0.01,
        p_transp_dom: float = 0.01,
        p_reg_dom: float = 0.01,
        n_dom_type_codons: int = 2,
    ):
        if any(len(d) != CODON_SIZE for d in start_codons):
            raise ValueError(f"Not all start codons are of length {CODON_SIZE}")
        if any(len(d) != CODON_SIZE for d in stop_codons):
            raise ValueError(f"Not all stop codons are of length {CODON_SIZE}")
        both = set(start_codons) & set(stop_codons)
        if both:
            raise ValueError(f"Overlapping start and stop codons: {','.join(str(d) for d in both)}")
        if p_catal_dom + p_transp_dom + p_reg_dom > 1.0:
            raise ValueError("p_catal_dom, p_transp_dom, p_reg_dom together must not be greater 1.0")

        self.start_codons = list(start_codons)
        self.stop_codons = list(stop_codons)
        self.dom_size = (n_dom_type_codons + 5) * CODON_SIZE
        self.dom_type_size = n_dom_type_codons * CODON_SIZE

        prefixes = codons(n=n_dom_type_codons, excl_codons=self.start_codons)
        random.shuffle(prefixes)
        n = len(prefixes)
        counts = (
            _n_of(p_catal_dom, n, "catalytic domains"),
            _n_of(p_transp_dom, n, "transporter domains"),
            _n_of(p_reg_dom, n, "allosteric domains"),
        )
        self.domain_types: dict[int, list[str]] = {}
        i = 0
        for dom_type, k in zip((1, 2, 3), counts):
            self.domain_types[dom_type] = prefixes[i : i + k]
            i += k
        self.domain_map = {seq: t for t, seqs in self.domain_types.items() for seq in seqs}

        stops = set(self.stop_codons)
        self.one_codon_map = {d: i + 1 for i, d in enumerate(c for c in codons(n=1) if c not in stops)}
        self.two_codon_map = {
            d: i + 1 for i, d in enumerate(c for c in codons(n=2) if c[:CODON_SIZE] not in stops)
        }
        self.idx_2_one_codon = {v: k for k, v in self.one_codon_map.items()}
        self.idx_2_two_codon = {v: k for k, v in self.two_codon_map.items()}

        self._tables = None
        self._tables_key: tuple | None = None

    # ------------------------------------------------------------------ native tables
    def _key(self) -> tuple:
        return (
            tuple(self.start_codons),
            tuple(self.stop_codons),
            id(self.domain_map),
            len(self.domain_map),
            id(self.one_codon_map),
            id(self.two_codon_map),
            self.dom_size,
            self.dom_type_size,
        )

    @property
    def tables(self):
        """Native translation tables (rebuilt if the codon lists or maps were replaced)."""
        key = self._key()
        if self._tables is None or key != self._tables_key:
            self._tables = native.host().TranslationTables(
                self.start_codons,
                self.stop_codons,
                self.domain_map,
                self.one_codon_map,
                self.two_codon_map,
                self.dom_size,
                self.dom_type_size,
            )
            self._tables_key = key
            self._device_luts = {}
        return self._tables

    def device_luts(self, device) -> dict:
        """The translation LUTs as tensors on ``device`` (cached per device)."""
        import torch

        tables = self.tables
        key = str(device)
        cache = self.__dict__.setdefault("_device_luts", {})
        if key not in cache:
            st, sp, oc, dt, tc = tables.luts()
            cache[key] = {
                "small": torch.from_numpy(np.concatenate([np.asarray(st), np.asarray(sp), np.asarray(oc)])).to(device),
                "is_start": torch.from_numpy(np.asarray(st)).to(device),
                "is_stop": torch.from_numpy(np.asarray(sp)).to(device),
                "one_codon": torch.from_numpy(np.asarray(oc)).to(device),
                "dom_type": torch.from_numpy(np.asarray(dt)).to(device),
                "two_codon": torch.from_numpy(np.asarray(tc)).to(device),
            }
        return cache[key]

    def __getstate__(self):
        state = self.__dict__.copy()
        state["_tables"] = None
        state["_tables_key"] = None
        state["_device_luts"] = {}
        state.pop("_hip_scratch", None)  # (device scratch of the translation launches)
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        # (a reference pickle has no native-table cache)
        self.__dict__.setdefault("_tables", None)
        self.__dict__.setdefault("_tables_key", None)
        self.__dict__.setdefault("_device_luts", {})

    # ------------------------------------------------------------------ API
    def translate_genomes(self, genomes: list[str]) -> list[list[ProteinSpecType]]:
        """Translate genomes into proteome specifications.

        Returns one list per genome of proteins ``(domains, cds_start, cds_end, is_fwd)`` where each
        domain is ``((dom_type, i0, i1, i2, i3), dom_start, dom_end)`` with CDS-relative offsets.
        Forward-strand proteins come first; reverse-strand coordinates index the reverse complement.
        """
        if len(genomes) < 1:
            return []
        return self.tables.translate_genomes(list(genomes))

    def _get_single_codons(self) -> list[str]:
        return [d for d in codons(n=1) if d not in self.stop_codons]

    def _get_double_codons(self) -> list[str]:
        return [d for d in codons(n=2) if d[:CODON_SIZE] not in self.stop_codons]
