"""Protein kinetics: token -> parameter maps, cell parameter tensors and the signal integrator.

Public surface and numerics follow the reference ``python/magicsoup/kinetics.py``:

* token maps (``kinetics.py:16-289``): Hill numbers, log-normal Km / Vmax weights, signs and the
  reaction / transporter / effector stoichiometry vectors, each with an ``inverse()`` used by the
  genome factories;
* dense per-cell parameters ``N, Nf, Nb, A`` (int32, (c, p, s)), ``Kmr`` (f32, (c, p, s)) and
  ``Kmf, Kmb, Vmax, Ke`` (f32, (c, p)) that users and tests may read and assign;
* ``integrate_signals`` = 3 parts with Vmax trimmed by 0.7 / 0.2 / 0.1, each with the
  negative-concentration guard and up to 4 equilibrium-damping iterations with a global early exit.

The hot paths are native: ``integrate_signals`` runs the fused kernel of ``csrc/hip/kinetics.hip`` on
GPU (``csrc/host/kinetics_host.cpp`` on CPU) and ``set_cell_params`` / ``set_cell_params_tokens``
run the fused parameter builder. The private ``_get_*`` / ``_multiply_signals`` helpers are kept as
plain-PyTorch specifications of each stage; they are the oracle the native kernels are tested
against, and they run when a subclass overrides them (e.g. to switch stages off in a test).
"""
from __future__ import annotations

import math
import os
import random
import weakref
from typing import Any

import numpy as np
import torch

from magicsoup_amd.constants import GAS_CONSTANT, ProteinSpecType, EPS as _EPS, MAX as _MAX, MIN as _MIN
from magicsoup_amd.models.containers import Chemistry, Molecule, Protein
from magicsoup_amd.ops import kinetics_ops

__all__ = ["Kinetics", "_EPS", "_MAX", "_MIN"]

_TRIMS = (0.7, 0.2, 0.1)
_INCREMENTS = (0.5, 0.25, 0.125, 0.0625)


class _HillMapFact:
    """Token -> Hill coefficient 1..5 with chances 16/31, 8/31, 4/31, 2/31, 1/31."""

    def __init__(self, max_token: int, device: str = "cpu", zero_value: int = 0):
        pool = [1] * 16 + [2] * 8 + [3] * 4 + [4] * 2 + [5]
        vals = [zero_value] + random.choices(pool, k=max_token)
        self.numbers = torch.tensor(vals, dtype=torch.int32, device=device)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return self.numbers[t]

    def inverse(self) -> dict[int, list[int]]:
        nums = self.numbers.cpu().tolist()
        return {h: [i for i, v in enumerate(nums) if v == h] for h in (1, 3, 5)}


class _LogNormWeightMapFact:
    """Token -> float drawn from a log-normal truncated to ``weight_range`` (token 0 -> NaN).

    mu is the mean of the log bounds and sigma the log range (reference kinetics.py:53-64).
    """

    def __init__(
        self,
        max_token: int,
        weight_range: tuple[float, float],
        device: str = "cpu",
        zero_value: float = math.nan,
    ):
        lo, hi = min(weight_range), max(weight_range)
        llo, lhi = math.log(lo), math.log(hi)
        mu, sig = (llo + lhi) / 2, lhi - llo
        vals = []
        for _ in range(max_token):
            v = math.exp(random.gauss(mu, sig))
            while not lo <= v <= hi:
                v = math.exp(random.gauss(mu, sig))
            vals.append(v)
        self.weights = torch.tensor([zero_value] + vals, dtype=torch.float32, device=device)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return self.weights[t]

    def inverse(self) -> dict[float, list[int]]:
        out: dict[float, list[int]] = {}
        for i, v in enumerate(self.weights.cpu().tolist()):
            if i > 0:
                out.setdefault(v, []).append(i)
        return out


class _SignMapFact:
    """Token -> +1 / -1 with equal chance (token 0 -> 0)."""

    def __init__(self, max_token: int, device: str = "cpu", zero_value: int = 0):
        vals = [zero_value] + random.choices([1, -1], k=max_token)
        self.signs = torch.tensor(vals, dtype=torch.int32, device=device)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return self.signs[t]

    def inverse(self) -> dict[bool, list[int]]:
        s = self.signs.cpu().tolist()
        return {True: [i for i, v in enumerate(s) if v == 1], False: [i for i, v in enumerate(s) if v == -1]}


class _VectorMapFact:
    """Token -> one of ``vectors`` (uniformly assigned); token 0 -> the zero vector."""

    def __init__(
        self,
        max_token: int,
        n_signals: int,
        vectors: list[list[int]],
        device: str = "cpu",
        zero_value: int = 0,
    ):
        M = torch.full((max_token + 1, n_signals), fill_value=zero_value, dtype=torch.int32)
        if len(vectors) > 0:
            if any(len(v) != n_signals for v in vectors):
                raise ValueError(f"Not all vectors have length of signal_size={n_signals}")
            if len(vectors) > max_token:
                raise ValueError(
                    f"There are max_token={max_token} and {len(vectors)} vectors."
                    " It is not possible to map all vectors"
                )
            if any(all(d == 0 for d in v) for v in vectors):
                raise ValueError(
                    "At least one vector includes only zeros."
                    " Each vector should contain at least one non-zero value."
                )
            picks = random.choices(range(len(vectors)), k=max_token)
            M[1:] = torch.tensor([vectors[i] for i in picks], dtype=torch.int32)
        self.M = M.to(device)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return self.M[t]


class _ReactionMapFact(_VectorMapFact):
    """Token -> stoichiometry vector (length 2m) of a chemistry reaction (intracellular half only)."""

    def __init__(
        self,
        molmap: dict[Molecule, int],
        reactions: list[tuple[list[Molecule], list[Molecule]]],
        max_token: int,
        device: str = "cpu",
        zero_value: int = 0,
    ):
        n_signals = 2 * len(molmap)
        vecs = [_stoich(molmap, subs, prods, n_signals) for subs, prods in reactions]
        super().__init__(max_token=max_token, n_signals=n_signals, vectors=vecs, device=device, zero_value=zero_value)

    def inverse(
        self,
        molmap: dict[Molecule, int],
        reactions: list[tuple[list[Molecule], list[Molecule]]],
        n_signals: int,
    ) -> dict[tuple[tuple[Molecule, ...], tuple[Molecule, ...]], list[int]]:
        M = self.M.cpu()
        out = {}
        for subs, prods in reactions:
            v = torch.tensor(_stoich(molmap, subs, prods, n_signals), dtype=M.dtype)
            out[(tuple(subs), tuple(prods))] = torch.argwhere((M == v).all(dim=1)).flatten().tolist()
        return out


def _stoich(molmap, subs, prods, n_signals) -> list[int]:
    v = [0] * n_signals
    for mol in subs:
        v[molmap[mol]] -= 1
    for mol in prods:
        v[molmap[mol]] += 1
    return v


class _TransporterMapFact(_VectorMapFact):
    """Token -> transport vector: -1 for the intracellular, +1 for the extracellular signal."""

    def __init__(self, n_molecules: int, max_token: int, device: str = "cpu", zero_value: int = 0):
        n = n_molecules
        vecs = [[-1 if j == i else (1 if j == i + n else 0) for j in range(2 * n)] for i in range(n)]
        super().__init__(max_token=max_token, n_signals=2 * n, vectors=vecs, device=device, zero_value=zero_value)

    def inverse(self, molecules: list[Molecule]) -> dict[Molecule, list[int]]:
        M = self.M.cpu()
        return {mol: torch.argwhere(M[:, i] != 0).flatten().tolist() for i, mol in enumerate(molecules)}


class _RegulatoryMapFact(_VectorMapFact):
    """Token -> one-hot effector signal (index >= m means extracellular / transmembrane)."""

    def __init__(self, n_molecules: int, max_token: int, device: str = "cpu", zero_value: int = 0):
        s = 2 * n_molecules
        vecs = [[1 if j == i else 0 for j in range(s)] for i in range(s)]
        super().__init__(max_token=max_token, n_signals=s, vectors=vecs, device=device, zero_value=zero_value)

    def inverse(self, molecules: list[Molecule]) -> dict[tuple[Molecule, bool], list[int]]:
        n = len(molecules)
        M = self.M.cpu()
        out = {}
        for i, mol in enumerate(molecules):
            out[(mol, False)] = torch.argwhere(M[:, i] != 0).flatten().tolist()
            out[(mol, True)] = torch.argwhere(M[:, i + n] != 0).flatten().tolist()
        return out


_PARAMS = ("Ke", "Kmf", "Kmb", "Kmr", "Vmax", "N", "Nf", "Nb", "A")
_I32_PARAMS = ("N", "Nf", "Nb", "A")
# integrator layout (GPU): "_W" (rows, P, s) packed int8x4 (N, Nf, Nb, A) words, "_Q" (rows, P, 4)
# (Vmax, Kmf, Kmb, Ke); derived from these API tensors, kept in the same row storage
_PACK_SRC = ("N", "Nf", "Nb", "A", "Vmax", "Kmf", "Kmb", "Ke")
_PACKED = ("_W", "_Q")
# compact GPU parameter storage (Kinetics._compact_store); MS_COMPACT_PARAMS=0 keeps all tensors
_COMPACT = os.environ.get("MS_COMPACT_PARAMS", "1") != "0"


def _spare_rows(n: int, row_bytes: int) -> int:
    """Spare parameter-storage rows kept beyond the n live ones: up to 3n within an 8 GiB budget,
    at least n / 8 (every rebuilt cell takes a fresh row; the spare count sets how many steps pass
    between row recycles, which cost one mark + compaction pass each)."""
    return max(n // 8, min(3 * n, (8 << 30) // max(row_bytes, 1)), 1024)


# ragged parameter records (csrc/hip/params.h): slot = offset | count << 32 | build width << 48
_REC_OFF_BITS = 32
_REC_CNT_BITS = 16
_REC_CNT_MASK = (1 << _REC_CNT_BITS) - 1
_MAX_PROTEINS = (1 << 15) - 1  # (the widths the host encodes stay below the int64 sign bit)


def _rec_code(off: int, cnt: int, width: int) -> int:
    return int(off) + (int(cnt) << _REC_OFF_BITS) + (int(width) << (_REC_OFF_BITS + _REC_CNT_BITS))


def _retire_t(t: torch.Tensor | None) -> None:
    """A storage tensor about to be dropped while queued work may still read it (see
    models/strings.py _retire)."""
    if t is not None and t.is_cuda:
        t.record_stream(torch.cuda.current_stream(t.device))


def _record_flag(kin):
    """Mapped host word the record assignment sets when records run out (a host build sized its
    reservation wrong: raised at the next integration, as the int8 overflow flag)."""
    from magicsoup_amd.ops import hip_ops

    sc = hip_ops._scratch(kin)
    f = getattr(sc, "rec_flag", None)
    if f is None:
        f = sc.rec_flag = hip_ops._HostFlag()
    return f


class Kinetics:
    """Protein work of all cells.

    Parameters:
        chemistry: Simulation chemistry.
        abs_temp: Absolute temperature (K); scales the equilibrium constants.
        km_range / vmax_range: Ranges of the log-normal Km (mM) / Vmax (mM/s) token weights.
        device: Device of all tensors (must match the world's).
        scalar_enc_size: Number of 1-codon tokens (``max(genetics.one_codon_map.values())``).
        vector_enc_size: Number of 2-codon tokens (``max(genetics.two_codon_map.values())``).

    Signals are the m intracellular molecules followed by the m extracellular ones (s = 2m).
    Cell parameters: ``Kmf, Kmb, Vmax, Ke`` (c, p); ``Kmr`` (c, p, s), already raised to the Hill
    exponent; ``N, Nf, Nb`` stoichiometry (net / forward / backward) and ``A`` allosteric Hill
    exponents (c, p, s, int32).
    """

    def __init__(
        self,
        chemistry: Chemistry,
        abs_temp: float = 310.0,
        km_range: tuple[float, float] = (1e-2, 100.0),
        vmax_range: tuple[float, float] = (1e-3, 100.0),
        device: str = "cpu",
        scalar_enc_size: int = 64 - 3,
        vector_enc_size: int = 4096 - 3 * 64,
    ):
        self.abs_temp = abs_temp
        self.device = device
        self.mol_names = [d.name for d in chemistry.molecules]
        self.mol_energies = torch.tensor(
            [d.energy for d in chemistry.molecules] * 2, dtype=torch.float32, device=device
        )
        s = 2 * len(chemistry.molecules)
        self.n_signals = s
        self.__dict__.update(_store_d={}, _slot=None, _ncells=0, _nrows=0)
        for name in _PARAMS:
            shape = (0, 0, s) if name in ("Kmr", "N", "Nf", "Nb", "A") else (0, 0)
            dt = torch.int32 if name in ("N", "Nf", "Nb", "A") else torch.float32
            setattr(self, name, torch.zeros(*shape, dtype=dt, device=device))

        mol_2_mi = {d: i for i, d in enumerate(chemistry.molecules)}
        self.km_map = _LogNormWeightMapFact(max_token=scalar_enc_size, weight_range=km_range, device=device)
        self.vmax_map = _LogNormWeightMapFact(max_token=scalar_enc_size, weight_range=vmax_range, device=device)
        self.sign_map = _SignMapFact(max_token=scalar_enc_size, device=device)
        self.hill_map = _HillMapFact(max_token=scalar_enc_size, device=device)
        self.reaction_map = _ReactionMapFact(
            molmap=mol_2_mi, reactions=chemistry.reactions, max_token=vector_enc_size, device=device
        )
        self.transport_map = _TransporterMapFact(
            n_molecules=len(chemistry.molecules), max_token=vector_enc_size, device=device
        )
        self.effector_map = _RegulatoryMapFact(
            n_molecules=len(chemistry.molecules), max_token=vector_enc_size, device=device
        )

        self.km_2_idxs = self.km_map.inverse()
        self.vmax_2_idxs = self.vmax_map.inverse()
        self.sign_2_idxs = self.sign_map.inverse()
        self.hill_2_idxs = self.hill_map.inverse()
        self.trnsp_2_idxs = self.transport_map.inverse(molecules=chemistry.molecules)
        self.regul_2_idxs = self.effector_map.inverse(molecules=chemistry.molecules)
        self.catal_2_idxs = self.reaction_map.inverse(
            molmap=mol_2_mi, reactions=chemistry.reactions, n_signals=s
        )
        self.last_masks: list[int] = []

    # ------------------------------------------------------------------ proteome views
    def get_proteome(self, proteome: list[ProteinSpecType]) -> list[Protein]:
        """Human-readable :class:`Protein` views of one translated proteome."""
        from magicsoup_amd.models.containers import CatalyticDomain, RegulatoryDomain, TransporterDomain

        mols = [Molecule.from_name(n) for n in self.mol_names]
        m = len(mols)
        vmax = self.vmax_map.weights.cpu().tolist()
        km = self.km_map.weights.cpu().tolist()
        signs = self.sign_map.signs.cpu().tolist()
        hills = self.hill_map.numbers.cpu().tolist()
        RM, TM, EM = (self.reaction_map.M.cpu(), self.transport_map.M.cpu(), self.effector_map.M.cpu())
        out = []
        for doms, cds_start, cds_end, is_fwd in proteome:
            views = []
            for (t, i0, i1, i2, i3), start, end in doms:
                sign = signs[i2]
                if t == 1:
                    vec = RM[i3].tolist()
                    lft, rgt = [], []
                    for mi, nv in enumerate(vec):
                        sn = nv * sign
                        (rgt if sn > 0 else lft).extend([mols[mi % m]] * abs(nv) if sn != 0 else [])
                    views.append(CatalyticDomain((lft, rgt), km=km[i1], vmax=vmax[i0], start=start, end=end))
                elif t == 2:
                    vec = TM[i3].tolist()
                    mi = next(i for i, d in enumerate(vec) if d != 0)
                    views.append(
                        TransporterDomain(
                            mols[mi % m], km=km[i1], vmax=vmax[i0], is_exporter=vec[mi] * sign < 0, start=start, end=end
                        )
                    )
                elif t == 3:
                    vec = EM[i3].tolist()
                    mi = next(i for i, d in enumerate(vec) if d != 0)
                    views.append(
                        RegulatoryDomain(
                            mols[mi % m],
                            hill=hills[i0],
                            km=km[i1],
                            is_inhibiting=vec[mi] * sign < 0,
                            is_transmembrane=mi >= m,
                            start=start,
                            end=end,
                        )
                    )
            out.append(Protein(domains=views, cds_start=cds_start, cds_end=cds_end, is_fwd=is_fwd))
        return out

    # ------------------------------------------------------------------ parameter building
    def set_cell_params(self, cell_idxs: list[int], proteomes: list[list[ProteinSpecType]]):
        """Derive and write the parameters of cells ``cell_idxs`` from translated proteomes.

        Rows are written in place into the current parameter tensors; proteins beyond a proteome's
        length get the padding values of the reference (Ke 1, Kmf = Kmb = EPS, Kmr 1, rest 0).
        """
        if len(cell_idxs) == 0:
            return
        tokens = self._collect_proteome_idxs(proteomes)
        self.set_cell_params_tokens(cell_idxs, tokens)

    def set_cell_params_tokens(self, cell_idxs, tokens: torch.Tensor, nprot: torch.Tensor | None = None):
        """Fused parameter build from dense tokens (n, P, D, 5) int32 for cells ``cell_idxs``;
        cells with ``nprot == 0`` (if given) are unset. On the GPU the cells take fresh records of
        their proteomes' size (cells may share records: a division's child its parent's)."""
        if tokens.size(1) > self._P():
            self.increase_max_proteins(int(tokens.size(1)))
        dev = self._store["Kmr"].device
        if dev.type == "cuda":
            self._sync()
            cells = torch.as_tensor(cell_idxs, device=dev).long().contiguous()
            if cells.numel() == 0:
                return
            tokens = tokens.to(device=dev, dtype=torch.int32).contiguous()
            roff, nprot = self._alloc_cells(cells, tokens, nprot)
            kinetics_ops.build_params(self, None, tokens, nprot=nprot, roff=roff)
            return
        rows = torch.as_tensor(cell_idxs, dtype=torch.int32)
        kinetics_ops.build_params(self, rows, tokens, nprot=nprot)

    def unset_cell_params(self, cell_idxs):
        """Zero all parameters of the given cells."""
        if isinstance(cell_idxs, list) and len(cell_idxs) == 0:
            return
        if self._slot_tensor() is not None:
            # shared rows: point the cells at the all-zero row
            cells = torch.as_tensor(cell_idxs, device=self._slot_tensor().device).long()
            if cells.numel() == 0:
                return
            self.__dict__["_slot"][cells] = self._zero_row()
            return
        rows = self._rows(cell_idxs)
        ok = self._pack_ok()
        for t in self._store.values():
            t[rows] = 0
        self._restamp(ok)

    def copy_cell_params(self, from_idxs, to_idxs):
        """Copy the parameters of cells ``from_idxs`` to cells ``to_idxs`` (sources are read before
        any destination is written, as with ``t[to] = t[fr]``)."""
        self._sync()
        self._copy_rows(from_idxs, to_idxs, disjoint=False)

    def _copy_rows(self, from_idxs, to_idxs, disjoint: bool) -> None:
        """On the GPU the destination cells share the source cells' storage rows (no parameter
        copy; rows are never written in place while in row-storage mode). ``disjoint`` is kept for
        callers that know no destination is also a source."""
        store = self._store
        dev = store["Kmr"].device
        if dev.type == "cuda":
            self._enter_slot_mode()
            slot = self.__dict__["_slot"]
            fr = torch.as_tensor(from_idxs, device=dev).long()
            to = torch.as_tensor(to_idxs, device=dev).long()
            slot[to] = slot[fr]
            return
        fr, to = self._rows(from_idxs), self._rows(to_idxs)
        ok = self._pack_ok()
        for t in store.values():
            t[to] = t[fr]
        self._restamp(ok)

    def append_shared(self, from_idxs: torch.Tensor, gathered: bool = False) -> None:
        """Append cells that share the parameter rows of cells ``from_idxs`` (children of a
        division inherit the parent's proteome; reference kinetics.py:646-665 copies the rows).
        GPU row storage only. ``gathered``: the world's clone gather already wrote the new entries
        (``slot_clone_pairs``)."""
        k = int(from_idxs.numel())
        if k == 0:
            return
        self._enter_slot_mode()
        d = self.__dict__
        slot = d["_slot"]
        new = self._slot_append(k)
        if not gathered:
            torch.index_select(slot, 0, from_idxs.long(), out=new)  # `slot`: the map before growing
        d["_ncells"] += k

    # ---- parameter storage ----
    # CPU (and a GPU world right after its dense tensors were read from Python): dense, cell-ordered
    # (c, p, s) / (c, p) tensors, as the reference keeps them (kinetics.py:399-409).
    #
    # GPU: ragged records (csrc/hip/params.h). Every protein of a cell is one record of a record pool
    # -- its packed stoichiometry words "_W" (s int32), "Kmr" (s fp32) and "_Q" (Vmax, Kmf, Kmb, Ke) --
    # and a cell owns a contiguous run of as many records as its proteome has proteins, named by one
    # int64 per cell (_slot: offset, count, build width). No cell is padded to the population's longest
    # proteome: a population of 500 nt genomes holds ~10 records per cell instead of the 45-160 protein
    # slots of a dense row, and widening the protein dimension moves nothing (_pmax is only a bound).
    # Records are written once: a rebuild takes fresh records from the device bump counter _rtop
    # (the genome pipeline's chains take theirs on the device, gp.hip), a division's child shares its
    # parent's, and removing cells only compacts the slot map. When the pool runs out the live records
    # are compacted into a fresh pool (_collect_records). The host keeps an upper bound _rtop_ub of the
    # device counter (worst cases added at issue, tightened from the chains' status words), so issuing
    # a build never waits for the device. Reading a parameter tensor from Python materialises the dense
    # tensors (records_to_dense: the reference's padding for a cell's missing proteins), which users
    # may modify in place; the next kernel use packs them back into records.
    @property
    def _store(self) -> dict[str, torch.Tensor]:
        return self.__dict__["_store_d"]

    def _P(self) -> int:
        d = self.__dict__
        if d.get("_slot") is not None:
            return int(d.get("_pmax", 0))
        store = self._store
        return int(store["Kmr"].size(1)) if "Kmr" in store and store["Kmr"].dim() == 3 else 0

    def _get_param(self, name: str) -> torch.Tensor:
        self._sync()
        self._materialize()
        t = self._store[name]
        n = self.__dict__["_ncells"]
        return t if t.size(0) == n else t[:n]

    def _set_param(self, name: str, value) -> None:
        d = self.__dict__
        if "_store_d" not in d:
            d["_store_d"], d["_slot"], d["_ncells"], d["_nrows"] = {}, None, 0, 0
        self._sync()
        self._materialize()
        self._drop_packed()
        t = torch.as_tensor(value)
        if not t.is_contiguous():
            t = t.contiguous()
        self._store[name] = t
        d["_ncells"] = d["_nrows"] = int(t.size(0))
        d.get("_spare", {}).pop(name, None)

    def _rows(self, cells):
        """Dense storage rows of cells (the dense layout is cell ordered)."""
        return cells

    def _slot_tensor(self) -> torch.Tensor | None:
        return self.__dict__["_slot"]

    def _enter_slot_mode(self) -> None:
        """GPU: switch from the dense layout to ragged records. The dense rows become records as they
        are (cell i's P proteins at records i * P .., a view: nothing is copied), so the parameters a
        user may have written are kept exactly; rebuilt cells then take records of their own size.
        The slot map lives in a capacity buffer (plus a spare of the same size for compactions), so
        the world moves it together with its per-cell columns in one row gather."""
        d = self.__dict__
        if d["_slot"] is not None:
            return
        store = self._store
        dev = store["Kmr"].device
        if dev.type != "cuda":
            return
        n = d["_ncells"]
        s = int(self.n_signals)
        if store["Kmr"].dim() == 3 and store["Kmr"].size(1) > 0:
            packed = self._packed_params()
            P, rows = int(packed["Kmr"].size(1)), int(packed["Kmr"].size(0))
            W = packed["_W"].reshape(rows * P, s)
            Q = packed["_Q"].reshape(rows * P, 4)
            K = packed["Kmr"].reshape(rows * P, s)
        else:
            P, rows = 0, 0
            W = torch.zeros(0, s, dtype=torch.int32, device=dev)
            Q = torch.zeros(0, 4, dtype=torch.float32, device=dev)
            K = torch.zeros(0, s, dtype=torch.float32, device=dev)
        if P > _MAX_PROTEINS:
            raise ValueError(f"a proteome of {P} proteins exceeds the record layout's {_MAX_PROTEINS}")
        store.clear()
        store.update({"_W": W, "_Q": Q, "Kmr": K})
        d.pop("_spare", None)
        self._slot_reserve(n, dev)
        buf = d["_slot_buf"]
        if P:
            torch.arange(n, device=dev, out=buf[:n])
            buf[:n].mul_(P).add_(_rec_code(0, P, P))
        else:
            buf[:n].zero_()
        d["_slot"] = buf[:n]
        d["_pmax"] = P
        d["_rtop"] = torch.full((1,), n * P, dtype=torch.int64, device=dev)
        d["_rtop_ub"] = n * P
        d.setdefault("_res_total", 0)
        d["_compact"] = True
        d["_free"] = None
        d.pop("_packed_stamp", None)

    def _slot_reserve(self, n: int, dev=None) -> None:
        """Capacity of the slot buffers >= n (keeps the live entries)."""
        d = self.__dict__
        buf = d.get("_slot_buf")
        if buf is not None and buf.numel() >= n:
            return
        dev = dev if dev is not None else d["_slot"].device
        cap = max(n, int((0 if buf is None else buf.numel()) * 1.5) + 1024)
        nb = torch.empty(cap, dtype=torch.int64, device=dev)
        cur = d.get("_slot")
        if cur is not None and cur.numel():
            nb[: cur.numel()] = cur
        d["_slot_buf"] = nb
        d["_slot_spare"] = torch.empty(cap, dtype=torch.int64, device=dev)
        if cur is not None:
            d["_slot"] = nb[: cur.numel()]

    def _slot_append(self, k: int) -> torch.Tensor:
        """Grow the live slot map by k entries; returns the view of the new entries."""
        d = self.__dict__
        n = int(d["_slot"].numel())
        self._slot_reserve(n + k)
        buf = d["_slot_buf"]
        d["_slot"] = buf[: n + k]
        return buf[n : n + k]

    def slot_compact_pairs(self, n: int) -> list:
        """(live map, spare rows) for a world's order-preserving row gather of ``n`` cells (empty
        when not in slot mode); adopt with ``remove_cell_params(..., gathered=True)``."""
        d = self.__dict__
        if d["_slot"] is None or d["_slot"].numel() != n:
            return []
        return [(d["_slot"], d["_slot_spare"][:n])]

    def slot_clone_pairs(self, n: int, k: int) -> list:
        """(map, map) over the first n + k entries for a world's clone gather of k new cells
        (children at rows n..); adopt with ``append_shared(..., gathered=True)``."""
        self._enter_slot_mode()
        d = self.__dict__
        if d["_slot"].numel() != n:
            return []
        self._slot_reserve(n + k)
        buf = d["_slot_buf"]
        return [(buf[: n + k], buf[: n + k])]

    def _sync(self) -> None:
        """Resolve pending device-pipeline updates of the owning world (no-op otherwise)."""
        ref = self.__dict__.get("_owner")
        w = ref() if ref is not None else None
        if w is not None and (w.__dict__.get("_gp_state") or w.__dict__.get("_deferred")
                              or w.__dict__.get("_count_pending") is not None):
            w._reconcile()

    def _zero_row(self) -> torch.Tensor:
        """The slot (int64 (1,), device) of a cell without parameters: 0 (no records; the dense view
        is all zero, as after unset_cell_params). Cells are pointed at it by filling their slots."""
        d = self.__dict__
        z = d.get("_zero_row_t")
        if z is None or z.device != self._store["Kmr"].device:
            z = d["_zero_row_t"] = torch.zeros(1, dtype=torch.int64, device=self._store["Kmr"].device)
        return z

    # -- record pool
    def _rec_cap(self) -> int:
        return int(self._store["Kmr"].size(0))

    def _row_limit(self) -> tuple[int, None]:
        """(record capacity of the pool, None): the device genome pipeline takes records below it."""
        return self._rec_cap(), None

    def _est_records(self) -> int:
        """Records a device chain reserves per rebuilt cell: twice the live mean proteome plus 8,
        at most the protein bound. A chain that needs more than the pool holds flags the cells it
        could not place (genome_pipeline: rebuilt on the host, which reserves exactly), and its
        status resets the host bound, so an estimate costs a rare host rebuild, never corruption;
        the worst case (the bound, 45-160 proteins) would size the pool for nothing."""
        d = self.__dict__
        P = max(self._P(), 1)
        mean = d.get("_mean_np")
        return P if mean is None else max(1, min(P, int(2 * mean) + 8))

    def _rows_available(self, k: int) -> bool:
        """Whether the records of k rebuilt cells (estimated, :meth:`_est_records`) fit below the
        capacity without a collection (slot mode)."""
        d = self.__dict__
        if d.get("_slot") is None:
            return False
        return d["_rtop_ub"] + k * self._est_records() <= self._rec_cap()

    def _reserve_rows(self, k: int, sync: bool = True, headroom: int = 0) -> int:
        """Room for the records of k rebuilt cells that a device chain takes with its own counter
        (magicsoup_amd.ops.genome_pipeline): the capacity is made for k + ``headroom`` cells (a
        collection or growth now, so that the next chains find their records without one), k cells'
        records are added to the host bound (per cell :meth:`_est_records`). ``sync=False``: the
        owner's pending state is not resolved first (a chain issued on a device count; the caller
        checked :meth:`_rows_available`). Returns the reservation mark the chain's status is adopted
        with (:meth:`_adopt_rtop`)."""
        self._enter_slot_mode()
        e = self._est_records()
        self._ensure_records((k + headroom) * e, sync=sync)
        return self._note_records(k * e)

    def _note_records(self, need: int) -> int:
        d = self.__dict__
        d["_rtop_ub"] += int(need)
        d["_res_total"] = d.get("_res_total", 0) + int(need)
        return d["_res_total"]

    def _adopt_rtop(self, value: int, mark: int | None) -> None:
        """A chain's status holds the device counter right after its records were taken: the host
        bound becomes that plus what was reserved since the chain was issued."""
        d = self.__dict__
        if d.get("_slot") is None or mark is None:
            return
        ub = int(value) + (d.get("_res_total", 0) - int(mark))
        if ub < d["_rtop_ub"]:
            d["_rtop_ub"] = ub

    def _ensure_records(self, need: int, sync: bool = True) -> None:
        """Room for ``need`` more records above the host bound of the counter: a read of the device
        counter (after resolving the owner's pending chains), then a collection / growth."""
        d = self.__dict__
        if d["_rtop_ub"] + need <= self._rec_cap():
            return
        if not sync:
            raise RuntimeError("parameter records: no room for a chain issued without synchronisation")
        self._sync()
        if d["_rtop_ub"] + need <= self._rec_cap():
            return
        d["_rtop_ub"] = int(d["_rtop"].item())
        if d["_rtop_ub"] + need <= self._rec_cap():
            return
        self._collect_records(need)

    def _collect_records(self, need: int) -> None:
        """Compact the live cells' records into a fresh pool (in cell order, a run per cell) with room
        for ``need`` more, growing it when less than about the live size would be left free. Cells
        that shared a run (a division's parent and child) get a copy each. Two synchronisations (the
        live count, the counter)."""
        from magicsoup_amd.ops import hip_ops

        d = self.__dict__
        store = self._store
        n = d["_ncells"]
        slot = d["_slot"]
        dev = slot.device
        s = int(self.n_signals)
        cnt = (slot >> _REC_OFF_BITS) & _REC_CNT_MASK
        ends = torch.cumsum(cnt, 0)
        live = int(ends[-1].item()) if n else 0
        cap = self._rec_cap()
        free_target = max(live, int(need), 1 << 16)
        new_cap = cap if live + need + free_target // 2 <= cap else int((live + need + free_target) * 1.25)
        new_cap = min(new_cap, (1 << _REC_OFF_BITS) - 1)  # (offsets the slot layout can name)
        if live + need > new_cap:
            raise RuntimeError(f"parameter records: {live + need} records exceed the slot layout's {new_cap}")
        W2 = torch.empty(new_cap, s, dtype=torch.int32, device=dev)
        Q2 = torch.empty(new_cap, 4, dtype=torch.float32, device=dev)
        K2 = torch.empty(new_cap, s, dtype=torch.float32, device=dev)
        out = d["_slot_spare"][:n]
        if n:
            new_off = (ends - cnt).contiguous()
            hip_ops._m().records_move(n, s, slot.data_ptr(), new_off.data_ptr(), store["_W"].data_ptr(),
                                      store["_Q"].data_ptr(), store["Kmr"].data_ptr(), W2.data_ptr(), Q2.data_ptr(),
                                      K2.data_ptr(), out.data_ptr(), hip_ops._stream())
        from magicsoup_amd.models.strings import _retire

        for t in (store["_W"], store["_Q"], store["Kmr"], slot):
            _retire(t)
        store.update({"_W": W2, "_Q": Q2, "Kmr": K2})
        d["_slot_buf"], d["_slot_spare"] = d["_slot_spare"], d["_slot_buf"]
        d["_slot"] = d["_slot_buf"][:n]
        d["_rtop"].fill_(live)
        d["_rtop_ub"] = live
        if n:
            d["_mean_np"] = live / n
        d["_collections"] = d.get("_collections", 0) + 1

    def _alloc_cells(self, cells: torch.Tensor, tokens: torch.Tensor, nprot: torch.Tensor | None) -> torch.Tensor:
        """Records for the rebuilt ``cells`` (their proteomes: ``nprot`` proteins each, or counted from
        the tokens): taken on the device in cell order by one scan launch, the cells' slots written.
        Returns the first record of each (int64, -1: no proteins) and the protein counts (int32)."""
        from magicsoup_amd.ops import hip_ops

        self._enter_slot_mode()
        d = self.__dict__
        dev = d["_slot"].device
        k = int(cells.numel())
        if nprot is None:
            nprot = (tokens[..., 0] != 0).any(dim=-1).sum(dim=-1)
        nprot = nprot.to(device=dev, dtype=torch.int32).contiguous()
        # the exact count (the translation that made the tokens synchronised already): the host
        # bound stays tight, and the pool is not sized for the batch's longest proteome per cell
        need = int(nprot.sum().item())
        if k:
            mean = d.get("_mean_np")
            d["_mean_np"] = need / k if mean is None else 0.5 * (mean + need / k)
        self._ensure_records(need)
        self._note_records(need)
        roff = torch.empty(k, dtype=torch.int64, device=dev)
        flag = _record_flag(self)
        hip_ops._m().assign_records(k, 0, nprot.data_ptr(), cells.data_ptr(), d["_slot"].data_ptr(),
                                    d["_rtop"].data_ptr(), self._rec_cap(), self._P(), roff.data_ptr(),
                                    flag.data_ptr(), hip_ops._stream())
        return roff, nprot

    def _kernel_params(self) -> dict[str, torch.Tensor]:
        """Storage tensors in kernel layout (contiguous int32 / float32), rows = capacity."""
        store = self._store
        for name, t in list(store.items()):
            want = torch.int32 if (name in _I32_PARAMS or name == "_W") else torch.float32
            if t.dtype != want or not t.is_contiguous():
                self._materialize()
                store[name] = store[name].to(want).contiguous()
        return store

    # ---- integrator layout (GPU) ----
    # "_W" / "_Q" are rebuilt from the API tensors whenever those were replaced or modified from
    # Python (detected through tensor identity + version counter); the GPU parameter build writes
    # the packed layout directly.
    def _pack_stamp(self):
        store = self.__dict__.get("_store_d", {})
        return tuple((weakref.ref(store[k]), store[k]._version) for k in _PACK_SRC if k in store)

    def _pack_ok(self) -> bool:
        d = self.__dict__
        if d.get("_compact"):
            return True  # the packed layout is the only one held (see _compact_store)
        st = d.get("_packed_stamp")
        store = d.get("_store_d", {})
        if st is None or any(k not in store for k in _PACKED) or len(st) != len(_PACK_SRC):
            return False
        return all(ref() is store[k] and ver == store[k]._version for (ref, ver), k in zip(st, _PACK_SRC))

    def _restamp(self, ok: bool) -> None:
        """Mark the packed layout current after an op that moved it together with the sources."""
        if ok:
            self.__dict__["_packed_stamp"] = self._pack_stamp()

    def _drop_packed(self) -> None:
        if self.__dict__.get("_compact"):
            self._expand_store()
        store = self.__dict__.get("_store_d", {})
        for k in _PACKED:
            store.pop(k, None)
            self.__dict__.get("_spare", {}).pop(k, None)
        self.__dict__.pop("_packed_stamp", None)

    def _packed_params(self) -> dict[str, torch.Tensor]:
        """Storage tensors including the integrator layout (GPU only); repacks if stale."""
        store = self._kernel_params()
        if self._pack_ok():
            return store
        from magicsoup_amd.ops import hip_ops

        # pack the live rows only, in cell order
        self._materialize()
        store = self._store
        self._drop_packed()
        N = store["N"]
        rows, P, s = int(N.size(0)), int(N.size(1)), int(N.size(2))
        store["_W"] = torch.zeros(rows, P, s, dtype=torch.int32, device=N.device)
        store["_Q"] = torch.zeros(rows, P, 4, dtype=torch.float32, device=N.device)
        hip_ops.pack_params(self, store, self.__dict__["_ncells"])
        self._restamp(True)
        return store

    def _compact_store(self) -> None:
        d = self.__dict__
        store = self._store
        if not all(k in store for k in _PACKED):
            return
        for k in _PACK_SRC:
            store.pop(k, None)
            d.get("_spare", {}).pop(k, None)
        d["_compact"] = True
        d.pop("_packed_stamp", None)

    def _expand_store(self) -> None:
        """Unpack the eight parameter tensors from a dense _W / _Q (same rows) and leave compact
        mode."""
        d = self.__dict__
        if not d.get("_compact"):
            return
        store = self._store
        W, Q = store["_W"], store["_Q"]
        store["N"] = ((W << 24) >> 24).contiguous()
        store["Nf"] = ((W >> 8) & 0xFF).contiguous()
        store["Nb"] = ((W >> 16) & 0xFF).contiguous()
        store["A"] = (W >> 24).contiguous()
        for i, k in enumerate(("Vmax", "Kmf", "Kmb", "Ke")):
            store[k] = Q[..., i].contiguous()
        d["_compact"] = False
        self._restamp(True)

    def _materialize(self, expand: bool = True) -> None:
        """Dense, cell-ordered tensors (leaves record mode): every cell's records, the build's padding
        for its missing proteins (records_to_dense). ``expand``: also unpack the eight API tensors
        from the packed words."""
        d = self.__dict__
        slot = d.get("_slot")
        if slot is None:
            if expand:
                self._expand_store()
            return
        from magicsoup_amd.ops import hip_ops

        n = d["_ncells"]
        P = self._P()
        store = self._store
        s = int(self.n_signals)
        dev = slot.device
        Wd = torch.empty(n, P, s, dtype=torch.int32, device=dev)
        Qd = torch.empty(n, P, 4, dtype=torch.float32, device=dev)
        Kd = torch.empty(n, P, s, dtype=torch.float32, device=dev)
        hip_ops._m().records_to_dense(n, P, s, slot.data_ptr(), store["_W"].data_ptr(), store["_Q"].data_ptr(),
                                      store["Kmr"].data_ptr(), Wd.data_ptr(), Qd.data_ptr(), Kd.data_ptr(),
                                      hip_ops._stream())
        for t in list(store.values()):
            _retire_t(t)
        store.clear()
        store.update({"_W": Wd, "_Q": Qd, "Kmr": Kd})
        for k in ("_spare", "_rtop", "_rtop_ub", "_pmax", "_free"):
            d.pop(k, None)
        d["_slot"] = None
        d["_nrows"] = n
        d["_compact"] = True
        d.pop("_packed_stamp", None)
        if expand:
            self._expand_store()

    def remove_cell_params(self, keep: torch.Tensor, removed: torch.Tensor | None = None, gathered: bool = False):
        """Keep only the cells where ``keep`` is true (bool mask (c,)) or listed (ascending index
        tensor), preserving their order. ``removed`` (optional) lists the other cells.
        ``gathered``: the world's compaction gather already wrote the kept map entries into the
        spare buffer (``slot_compact_pairs``)."""
        self._sync()
        idx = torch.nonzero(keep).flatten() if keep.dtype == torch.bool else keep.to(torch.long)
        d = self.__dict__
        k = int(idx.numel())
        if idx.is_cuda:
            # only the slot map is compacted; the records of removed cells (possibly shared with
            # survivors) stay until the next collection
            if gathered and d["_slot"] is not None:
                d["_slot_buf"], d["_slot_spare"] = d["_slot_spare"], d["_slot_buf"]
            else:
                self._enter_slot_mode()
                torch.index_select(d["_slot"], 0, idx, out=d["_slot_spare"][:k])
                d["_slot_buf"], d["_slot_spare"] = d["_slot_spare"], d["_slot_buf"]
            d["_slot"] = d["_slot_buf"][:k]
            d["_ncells"] = k
            return
        self._materialize()
        ok = self._pack_ok()
        spare = d.setdefault("_spare", {})
        store = self._store
        n = d["_ncells"]
        for name, t in list(store.items()):
            sp = spare.get(name)
            if sp is None or sp.size(0) < max(k, 1) or sp.shape[1:] != t.shape[1:] or sp.dtype != t.dtype:
                sp = torch.empty(max(k, t.size(0)), *t.shape[1:], dtype=t.dtype, device=t.device)
            torch.index_select(t[:n], 0, idx, out=sp[:k])
            spare[name], store[name] = t, sp
        d["_ncells"] = d["_nrows"] = k
        self._restamp(ok)

    def reserve_cells(self, n: int) -> None:
        """Room for ``n`` cells allocated at once (no-op before the first proteome fixed the protein
        dimension). Record pool: three times the live cells' mean proteome per cell (a collection
        runs when garbage -- replaced and dead cells' records -- fills the rest); dense layout: rows
        plus the usual spare. Growing a large population in batches otherwise re-allocates the storage
        repeatedly with the old and the new copy alive together."""
        store = self._store
        if not store or self._P() == 0:
            return
        d = self.__dict__
        if d.get("_slot") is not None:
            self._sync()
            slot = d["_slot"]
            live = int(((slot >> _REC_OFF_BITS) & _REC_CNT_MASK).sum().item()) if slot.numel() else 0
            per = max(live / max(slot.numel(), 1), 4.0)
            want = int(3 * n * per) + (1 << 16)
            if want > self._rec_cap():
                self._grow_records(want)
            return
        cap = min(int(t.size(0)) for t in store.values())
        row_bytes = sum(t[:1].numel() * t.element_size() for t in store.values())
        want = n + _spare_rows(n, row_bytes)
        if want <= cap:
            return
        self._sync()
        ok = self._pack_ok()
        for name, t in list(store.items()):
            nb = torch.empty(want, *t.shape[1:], dtype=t.dtype, device=t.device)
            nb[:cap] = t[:cap]
            store[name] = nb
        self.__dict__.pop("_spare", None)
        self._restamp(ok)

    def _grow_records(self, cap: int) -> None:
        """A larger record pool: the records below the device counter are copied as they are."""
        d = self.__dict__
        store = self._store
        top = int(d["_rtop"].item())
        for name in ("_W", "_Q", "Kmr"):
            t = store[name]
            nb = torch.empty(cap, *t.shape[1:], dtype=t.dtype, device=t.device)
            if top:
                nb[:top] = t[:top]
            _retire_t(t)
            store[name] = nb
        d["_rtop_ub"] = top

    def increase_max_cells(self, by_n: int, zero: bool = True):
        """Append ``by_n`` cells (parameters zero-filled unless the caller writes them all)."""
        if by_n <= 0:
            return
        d = self.__dict__
        store = self._store
        if d["_slot"] is not None:
            # record storage: the new cells have no records (slot 0) until a build gives them some
            self._slot_append(by_n).zero_()
            d["_ncells"] += by_n
            return
        if store["Kmr"].device.type == "cuda" and d["_ncells"] == 0 and self._P() == 0:
            # a fresh GPU world: record storage from the start (no dense rows for the population)
            self._enter_slot_mode()
            return self.increase_max_cells(by_n, zero)
        cap = min(int(t.size(0)) for t in store.values())
        ok = self._pack_ok()
        n = d["_ncells"]
        if n + by_n > cap:
            new_cap = max(n + by_n, int(cap * 1.5) + 64)
            for name, t in list(store.items()):
                nb = torch.empty(new_cap, *t.shape[1:], dtype=t.dtype, device=t.device)
                nb[:n] = t[:n]
                store[name] = nb
            d.pop("_spare", None)
        d["_nrows"] = n + by_n
        d["_ncells"] = n + by_n
        if zero:
            for t in store.values():
                t[n : n + by_n].zero_()
        self._restamp(ok)

    def increase_max_proteins(self, max_n: int):
        """Grow the protein dimension of every parameter tensor to ``max_n`` (zero-filled). On the
        GPU only the bound grows: records are per protein, nothing moves (the dense view shows the
        new proteins as zeros, as the reference's widened tensors, kinetics.py:705-723)."""
        if max_n <= self._P():
            return
        self._sync()
        store = self._store
        if store["Kmr"].device.type == "cuda":
            if max_n > _MAX_PROTEINS:
                raise ValueError(f"a proteome of {max_n} proteins exceeds the record layout's {_MAX_PROTEINS}")
            self._enter_slot_mode()
            self.__dict__["_pmax"] = int(max_n)
            return
        self._materialize()
        ok = self._pack_ok()
        n = self.__dict__["_ncells"]
        for name, t in list(store.items()):
            t = t[:n]
            z = torch.zeros(n, max_n - t.size(1), *t.shape[2:], dtype=t.dtype, device=t.device)
            store[name] = torch.cat([t, z], dim=1)
        self.__dict__["_nrows"] = n
        self.__dict__.pop("_spare", None)
        self._restamp(ok)

    def _to_device(self, dev: torch.device) -> None:
        self._sync()
        self._materialize()
        self._drop_packed()
        n = self.__dict__["_ncells"]
        for name, t in list(self._store.items()):
            self._store[name] = t[:n].to(dev)
        self.__dict__["_nrows"] = n
        for k in ("_spare", "_slot_buf", "_slot_spare", "_zero_row_t"):
            self.__dict__.pop(k, None)

    # ------------------------------------------------------------------ integration
    def integrate_signals(self, X: torch.Tensor, _reduce_mask=None) -> torch.Tensor:
        """Let all proteins work for one time step.

        Parameters:
            X: Signals (c, s): intracellular molecules then the extracellular molecules of each
                cell's pixel. Must be >= 0.

        Returns:
            Updated signals (c, s) as a new tensor.
        """
        self._sync()
        if self._stages_overridden():
            for trim in _TRIMS:
                X = self._integrate_signals_part(adj_vmax=(self.Vmax * trim).clamp(0.0), X0=X)
            return X
        out = X.to(torch.float32).contiguous().clone()
        self.last_masks = kinetics_ops.integrate(
            self, out, trims=_TRIMS, n_iters=len(_INCREMENTS), reduce_mask=_reduce_mask
        )
        return out

    def _stages_overridden(self) -> bool:
        cls = type(self)
        return any(
            getattr(cls, name) is not getattr(Kinetics, name)
            for name in (
                "_integrate_signals_part",
                "_get_velocities",
                "_get_equilibrium_adjusted_x",
                "_get_negative_adjusted_nv",
                "_get_quotient",
                "_multiply_signals",
            )
        )

    # ---- PyTorch specifications of each stage (oracle for the native kernels) ----
    def _integrate_signals_part(self, adj_vmax: torch.Tensor, X0: torch.Tensor) -> torch.Tensor:
        V = self._get_velocities(X=X0, Vmax=adj_vmax)
        NV = self.N.float() * V.unsqueeze(2)
        NV_adj = self._get_negative_adjusted_nv(NV=NV, X=X0)
        X1 = (X0 + NV_adj.sum(1)).clamp(min=0.0)
        return self._get_equilibrium_adjusted_x(X0=X0, X1=X1, NV=NV_adj, V=V)

    def _get_velocities(self, X: torch.Tensor, Vmax: torch.Tensor) -> torch.Tensor:
        kf, f_on = self._multiply_signals(X=X, N=self.Nf)
        kf = torch.where(f_on, kf / self.Kmf, 0.0)
        kf = torch.where(kf.isinf(), _MAX, kf)
        kb, b_on = self._multiply_signals(X=X, N=self.Nb)
        kb = torch.where(b_on, kb / self.Kmb, 0.0)
        kb = torch.where(kb.isinf(), _MAX, kb)
        a_cat = (kf - kb) / (1 + kf + kb)

        is_reg = self.A != 0
        x_reg = is_reg.float() * X.unsqueeze(1)
        a = torch.pow(x_reg, self.A)
        a = a / (a + self.Kmr)
        a = torch.where(a.isnan() | ~is_reg, 1.0, a)
        a_reg = torch.prod(a, 2)
        a_reg = torch.where(a_reg.isinf(), _MAX, a_reg)
        return (a_cat * Vmax * a_reg).clamp(_MIN, _MAX)

    def _get_equilibrium_adjusted_x(
        self, X0: torch.Tensor, X1: torch.Tensor, NV: torch.Tensor, V: torch.Tensor
    ) -> torch.Tensor:
        has_impact = V.abs() > 0.1
        is_fwd = V > 0.0
        F = torch.ones_like(V)
        hi_t, lo_t = 1.5, 1 / 1.5
        for inc in _INCREMENTS:
            QKe = self._get_quotient(X=X1) / self.Ke
            low = torch.where(is_fwd, QKe < lo_t, QKe > hi_t) & ~(is_fwd & (F == 1.0))
            high = torch.where(is_fwd, QKe > hi_t, QKe < lo_t) & ~(~is_fwd & (F == 0.0))
            if not torch.any((low | high) & has_impact):
                return X1
            F = (F - inc * high.float() + inc * low.float()).clamp(0.0, 1.0)
            X1 = (X0 + torch.einsum("cps,cp->cs", NV, F)).clamp(min=0.0)
        return X1

    def _get_negative_adjusted_nv(self, NV: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
        F = X / (-NV).clamp(min=0.0).sum(1)
        F = torch.where(F > 1.0, 1.0, F)
        removing = NV < 0.0
        F_prot = torch.where(removing, F.unsqueeze(1), 1.0)
        return NV * F_prot.min(dim=2).values.unsqueeze(2)

    def _get_quotient(self, X: torch.Tensor) -> torch.Tensor:
        prods, p_on = self._multiply_signals(X=X, N=self.Nb)
        subs, s_on = self._multiply_signals(X=X, N=self.Nf)
        prods = torch.where(p_on, prods, 0.0)
        subs = torch.where(s_on, subs, 0.0)
        return (prods / subs).clamp(min=_EPS, max=_MAX).nan_to_num(1.0)

    def _multiply_signals(self, X: torch.Tensor, N: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        on = N > 0
        x = on.float() * X.unsqueeze(1)
        xx = torch.prod(torch.pow(x, N), 2)
        xx = torch.where(xx.isnan() | (xx < 0.0), 0.0, xx)
        xx = torch.where(xx.isinf(), _MAX, xx)
        return xx, on.any(dim=2)

    # ------------------------------------------------------------------ helpers
    def _collect_proteome_idxs(self, proteomes: list[list[ProteinSpecType]]) -> torch.Tensor:
        """Dense int32 tokens (n, P, D, 5) of proteome specs (P >= 1, D >= 1)."""
        n = len(proteomes)
        P = max([len(p) for p in proteomes] + [1])
        D = max([len(doms) for p in proteomes for doms, *_ in p] + [1])
        arr = np.zeros((n, P, D, 5), dtype=np.int32)
        for ci, prots in enumerate(proteomes):
            for pi, (doms, *_) in enumerate(prots):
                for di, (spec, *_) in enumerate(doms):
                    arr[ci, pi, di] = spec
        return torch.from_numpy(arr)

    def __getstate__(self):
        self._sync()
        self._materialize()
        state = self.__dict__.copy()
        state["last_masks"] = []
        for k in ("_spare", "_hip_scratch", "_owner", "_lut_cache", "_slot_buf", "_slot_spare", "_free", "_zero_row_t",
                  "_rtop", "_rtop_ub", "_pmax"):
            state.pop(k, None)
        n = state["_ncells"]
        state["_store_d"] = {k: v[:n].clone() for k, v in self._store.items() if k not in _PACKED}
        state.pop("_packed_stamp", None)
        state["_nrows"] = n
        return state

    def __setstate__(self, state):
        if "_store_d" not in state and "N" in state:
            # a reference pickle (magicsoup.kinetics.Kinetics, kinetics.py:390-460)
            from magicsoup_amd.utils.checkpoint import reference_kinetics_state

            state = reference_kinetics_state(state)
        self.__dict__.update(state)

    def _i32_tensor(self, d: Any) -> torch.Tensor:
        return torch.tensor(d, device=self.device, dtype=torch.int32)

    def _f32_tensor(self, d: Any) -> torch.Tensor:
        return torch.tensor(d, device=self.device, dtype=torch.float32)


def _param_property(name: str) -> property:
    def get(self):
        return self._get_param(name)

    def set(self, value):
        self._set_param(name, value)

    return property(get, set, doc=f"Cell parameter tensor ``{name}`` (dense, in cell order).")


for _name in _PARAMS:
    setattr(Kinetics, _name, _param_property(_name))
