"""Sync-free genome updates on the GPU: ``mutate_cells()`` / ``recombinate_cells()`` (all cells).

The reference API returns nothing from these two operations (``world.py:689-745``), so nothing
forces the host to learn how many genomes changed. Here the whole chain stays on the device:

    draw event counts -> select the changed genomes (count kept on the device) -> apply
    -> commit to the genome arena -> translate -> fresh parameter rows -> parameter build

Every kernel after the selection strides over the device-side count (``dn`` arguments in
``csrc/hip``), so the host issues the chain without a synchronisation and runs ahead into the next
operations while the GPU works. What the host cannot rule out in advance raises flag bits instead:

* a result longer than the genome pool's length bound (``PoolArena.width``, what the calls' scratch
  rows are sized for), or one that finds the pool full, is not committed (``arena_scatter``); every
  later pipeline op of the same pending chain then does nothing (its count kernel sees the flag)
  and is *replayed* at reconcile time with its original RNG stream, after the bound was raised /
  the pool collected and the result committed -- exactly the sequential outcome;
* a proteome with more proteins than the parameter storage holds, more domains than the token
  slots, or a genome too long for the LDS translation pass, and parameter rows running out
  (``gp_check_assign_kernel``): the affected cells are rebuilt on the synchronous path.

:func:`reconcile` resolves all of this; the World calls it before every op that reads genomes or
parameters, changes cells or positions, or allocates rows (and the Kinetics object before any host
access to its parameters), so results never depend on which path ran. Event counts are capped at
``K_CAP`` per genome; the pipeline is only used when the expected count is far below that.

Disable with ``MS_SYNC_GENETICS=1`` (always the synchronous path).
"""
from __future__ import annotations

import math
import os

import torch

from magicsoup_amd.ops import hip_ops
from magicsoup_amd.ops.hip_ops import _m, _p, _rng, _scratch, _stream
from magicsoup_amd.ops.streams import NEvent

K_CAP = 32  # event-count cap per genome (P(Poisson(lam <= 1) > 32) < 1e-35)
D_CAP = 12  # domain slots per protein in the speculative token layout
# protein slots per cell in that layout: the kinetics' protein bound up to this (a long evolving run's
# few giant proteomes -- thousands of proteins -- would otherwise size every chain cell's token rows;
# the cells past it are listed and rebuilt on the host, gp.hip gp_check_assign_kernel)
P_CAP = 1024
# scratch bytes one call may take (its blob: result rows of the length bound, token rows, long-genome
# translation slots); a call past it takes the synchronous path, which works in chunks -- a long
# evolving run's length bound of 10^6 nt priced a merged chain at 70 GB
_BLOB_MAX = int(os.environ.get("MS_GP_BLOB_MAX", 8 << 30))
N_CAP = 8192  # genomes per pipeline call (the expected count is kept <= N_CAP / 4)
# largest Poisson mean of events per genome (rate x the genome length bound) a pipeline call takes:
# the per-genome event count is capped at K_CAP, and P(Poisson(4) > 32) < 1e-18
LAM_MAX = 4.0


def _cap(expected: float, limit: int) -> int:
    """Buffer / grid capacity of a call: far above the expected count (a count above it makes the
    call a no-op that reconcile replays on the synchronous path, see cap_skip), far below N_CAP
    for small rates, so the launches after the selection stay small."""
    return max(1, min(limit, int(8 * expected) + 256))


def _pair_cap(n: int, expected: float, extra) -> int | None:
    """Pair capacity of a recombination call over ``n`` cells whose pair count has the (worst-case)
    mean ``expected``; None if the call must not be issued. A count above the capacity makes the call
    a no-op that reconcile replays on the synchronous path -- except for a decomposed world's call
    carrying strip-boundary results (``extra``), which the replay cannot reproduce: such a call is
    issued only while its capacity clears the mean by 8 standard deviations (a skip then has a
    probability below 1e-15); beyond, the caller issues the recombination on its own."""
    limit = min(n, N_CAP) // 2
    if extra is not None and expected + 8.0 * math.sqrt(expected) + 64 > limit:
        return None
    return _cap(expected, limit)
# flag bits (select.hip DevFlag, mutations.hip kGp*)
_F_TRANSLATE, _F_CAPACITY, _F_ROWS, _F_WIDTH, _F_SKIPPED, _F_PARTIAL = 1, 2, 4, 8, 16, 32
_SEL_I32POS, _SEL_SET = 2, 0


_SYNC_ENV = os.environ.get("MS_SYNC_GENETICS") == "1"


def enabled(world) -> bool:
    if _SYNC_ENV:
        return False
    return bool(world.__dict__["_molmap"].is_cuda)  # GPU worlds (single map or strip of a decomposed one)


class _StatusSlot:
    """int64[4] in the extension's pinned status ring (valid once the call's event completed)."""

    __slots__ = ("vals", "_slot")

    def __init__(self, slot: int):
        self.vals = None
        self._slot = slot

    def __getitem__(self, i: int) -> int:
        if self.vals is None:
            self.vals = _m().status_read(self._slot)
        return self.vals[i]


class _Pending:
    """One issued pipeline call: what reconcile needs to resolve it."""

    __slots__ = ("kind", "args", "rng", "cells", "host", "event", "replay")

    def __init__(self, kind, args, rng, cells, host, event, replay):
        self.kind, self.args, self.rng, self.cells = kind, args, rng, cells
        self.host, self.event, self.replay = host, event, replay


def _state(world) -> dict:
    st = world.__dict__.get("_gp_state")
    if st is None:
        st = world.__dict__["_gp_state"] = {"pending": []}
    return st


def _cache(world) -> dict:
    """Per-world cache of the call descriptors (dropped with the world's pickled state)."""
    c = world.__dict__.get("_gp_cache")
    if c is None:
        c = world.__dict__["_gp_cache"] = {}
    return c


def _bufs(world, kind: str) -> dict:
    c = _cache(world)
    b = c.get(kind)
    if b is None:
        sc = _scratch(world)
        dev = world._genomes.data.device
        b = c[kind] = {
            "cnt": sc.get(f"gp_cnt_{kind}", 2, torch.int32, dev),
            "cnt2": sc.get(f"gp_cnt2_{kind}", 2, torch.int32, dev),
            "opflags": sc.get(f"gp_opflags_{kind}", 1, torch.int32, dev),
            "gflags": sc.get("gp_gflags", 1, torch.int32, dev),
            "d_rows": sc.get("gp_rows", 1, torch.int64, dev),
        }
    return b


def _nt(world, n: int, L: int) -> int:
    """Upper bound of the live genomes' total length for a call's expected counts: n genomes at the
    length bound, or the pool's used bytes (every live genome lies below its top). A long evolving
    run's few giant genomes raise the bound L a hundredfold over the typical genome, which priced
    every call of such a population off the pipeline."""
    return min(n * L, max(int(world._genomes.top_ub), 0))


def _blob_ok(world, L: int, sizes) -> bool:
    """The call's scratch (``sizes()``: gp_blob_bytes / gp_evolve_union_bytes of its parts) within
    _BLOB_MAX. Length bounds up to 16 Ki nt with token rows of up to 256 proteins stay below ~5 GB
    whatever the capacities (N_CAP), so the common case skips the native size calls (host time of
    small, host-bound configs)."""
    if _BLOB_MAX >= (8 << 30) and L <= 16384 and _token_p(world) <= 256:
        return True
    return sum(int(b) for b in sizes()) <= _BLOB_MAX


def _token_p(world) -> int:
    """Protein slots per cell of the chain's token layout (the _kin_desc bound)."""
    return min(world.kinetics._P(), P_CAP)


def _usable(world, expected: float, limit: float = N_CAP / 4) -> bool:
    return enabled(world) and expected <= limit


def _prepare_records(world, cells: int, sync: bool = True, headroom: int = 0) -> None:
    """Room in the kinetics' record pool for the parameters of a call's (at most) ``cells`` rebuilt
    cells, made BEFORE the call reads any world state: when the pool is short this resolves the
    pending chains and collects the records (a reconcile can change the population, the arena's
    length bound, ...), so the call must size itself afterwards."""
    _state(world)["res_mark"] = world.kinetics._reserve_rows(int(cells), sync=sync, headroom=headroom)


def _begin(world, kind: str) -> dict:
    """Per-call device state. A pending call of the same kind is resolved first (its scratch is
    reused); with nothing pending the shared flags are reset. (The call made room for its records
    first: _prepare_records.)"""
    st = _state(world)
    if st["pending"] and any(pd.kind == kind for pd in st["pending"]):
        reconcile(world)
    kin = world.kinetics
    b = _bufs(world, kind)
    kin._enter_slot_mode()
    fresh = not st["pending"]
    # (-1: the chain takes parameter records from the kinetics' own device counter, gp.hip)
    _m().gp_begin(_arena_desc(world, b), fresh, -1, _stream())
    return b


def _arena_desc(world, b: dict):
    """C++ descriptor of the genome pool and this call's device counters (gp.hip GpArena)."""
    a = b.get("desc")
    if a is None:
        a = b["desc"] = _m().GpArena()
        a.cnt, a.cnt2, a.opflags, a.gflags = _p(b["cnt"]), _p(b["cnt2"]), _p(b["opflags"]), _p(b["gflags"])
    # the record counter of the kinetics' ragged parameter storage (reported in the status slots)
    rtop = world.kinetics.__dict__.get("_rtop")
    a.d_rows = rtop.data_ptr() if rtop is not None else _p(b["d_rows"])
    arena = world._genomes
    a.data, a.lens, a.width, a.n = arena.data.data_ptr(), arena.lens.data_ptr(), arena.width, arena.n
    a.off, a.top, a.pool_cap = arena.off.data_ptr(), arena.top.data_ptr(), arena.pool_cap
    return a


def _r16(n: int) -> int:
    return (int(n) + 15) // 16 * 16


def _room(world, need: int) -> None:
    """Pool space for a call's worst case of committed results (every selected result as long as
    its scratch row); counted into the host bound of the device counter."""
    arena = world._genomes
    arena.ensure(need)
    arena.top_ub += need


def _gen_desc(world, dev):
    luts = world.genetics.device_luts(dev)
    c = _cache(world)
    hit = c.get("gen")
    if hit is not None and hit[0] is luts:
        return hit[1]
    g = _m().GpGen()
    tables = world.genetics.tables
    g.small, g.dom_type, g.two_codon = _p(luts["small"]), _p(luts["dom_type"]), _p(luts["two_codon"])
    g.dt_entries, g.dom_size, g.dom_type_size = int(luts["dom_type"].numel()), tables.dom_size, tables.dom_type_size
    c["gen"] = (luts, g)
    return g


def _kin_desc(world, dev):
    """Ragged parameter records (kernel layout, csrc/hip/params.h), token LUTs and the cell ->
    records map. Rebuilt only when the storage changed; the slot map pointer (swapped by every
    compaction) and the protein bound are refreshed on each call."""
    kin = world.kinetics
    kin._enter_slot_mode()
    store = kin._kernel_params()
    rec_cap = kin._rec_cap()
    key = (store["Kmr"].data_ptr(), store["_W"].data_ptr(), store["_Q"].data_ptr(), rec_cap,
           kin.__dict__["_rtop"].data_ptr(), float(kin.abs_temp), id(store), int(kin.n_signals))
    c = _cache(world)
    hit = c.get("kin")
    if hit is not None and hit[0] == key:
        k = hit[1]
    else:
        from magicsoup_amd.constants import GAS_CONSTANT
        from magicsoup_amd.ops.kinetics_ops import build_luts

        lu = build_luts(kin, dev)
        k = _m().GpKin()
        k.Kmr, k.W, k.Q, k.overflow = _p(store["Kmr"]), _p(store["_W"]), _p(store["_Q"]), _p(hip_ops._overflow_flag(kin))
        k.rtop, k.rec_cap = kin.__dict__["_rtop"].data_ptr(), rec_cap
        k.s = int(kin.n_signals)
        k.vmax, k.km, k.signs, k.hills = _p(lu["vmax"]), _p(lu["km"]), _p(lu["signs"]), _p(lu["hills"])
        k.react, k.trnsp, k.eff, k.energies = _p(lu["react"]), _p(lu["trnsp"]), _p(lu["eff"]), _p(lu["energies"])
        k.nw, k.nk, k.nsg, k.nh = lu["vmax"].numel(), lu["km"].numel(), lu["signs"].numel(), lu["hills"].numel()
        k.nv = int(lu["react"].size(0))
        k.abs_temp, k.gas = float(kin.abs_temp), float(GAS_CONSTANT)
        # the LUT tensors stay referenced by the cache entry while their pointers are in use
        c["kin"] = (key, k, lu)
    k.P = min(kin._P(), P_CAP)
    k.slot = kin._slot_tensor().data_ptr()
    return k


def _blob(world, kind: str, nbytes: int, dev) -> torch.Tensor:
    """The call's scratch blob; grown with 25 % headroom so that a slowly growing population does
    not re-allocate it every few steps."""
    sc = _scratch(world)
    name = f"gp_blob_{kind}"
    t = sc.bufs.get(name)
    if t is None or t.numel() < nbytes:
        sc.bufs[name] = t = torch.empty(nbytes + nbytes // 4, dtype=torch.uint8, device=dev)
    return t


_ES = {torch.uint8: 1, torch.int32: 4, torch.int64: 8}


def _view(blob: torch.Tensor, off: int, n: int, dtype) -> torch.Tensor:
    return blob[off : off + n * _ES[dtype]].view(dtype)


class _Replay:
    """What reconcile needs to re-commit a call's results (views into the call's scratch blob,
    made only when needed)."""

    __slots__ = ("blob", "lay", "n", "mark", "gen", "direct", "rows_key")

    def __init__(self, blob, lay, n, rows_key, mark=None, gen=0, direct=False):
        self.blob, self.lay, self.n, self.rows_key = blob, lay, n, rows_key
        self.mark, self.gen, self.direct = mark, gen, direct

    def views(self):
        lay, n, b = self.lay, self.n, self.blob
        return (_view(b, lay[self.rows_key], n, torch.int64), _view(b, lay["out"], n * lay["out_w"], torch.uint8),
                lay["out_w"], _view(b, lay["out_len"], n, torch.int32))


def _record(world, kind: str, args: tuple, rng: tuple, cells, slot: int, replay: dict) -> None:
    """Record an issued pipeline call as pending (its status lands in pinned slot ``slot``)."""
    ev = NEvent().record()
    _state(world)["pending"].append(_Pending(kind, args, rng, cells, _StatusSlot(slot), ev, replay))
    world._genomes.version += 1


def point_mutations(world, p: float, p_indel: float, p_del: float) -> bool:
    """Device-pipeline ``mutate_cells()`` over all cells (one C++ call issuing the chain, gp.hip);
    False if this call should take the synchronous path instead."""
    arena = world._genomes
    if arena.n == 0:
        return True
    if not enabled(world):
        return False
    # (the call's capacity at the current state: the record reservation's size; everything is
    # re-read after it)
    _prepare_records(world, _cap(p * _nt(world, arena.n, int(arena.width)), min(arena.n, N_CAP)))
    n = arena.n
    L = int(arena.width)  # every genome fits its row
    exp_mut = p * _nt(world, n, L)
    if p * L > LAM_MAX or not _usable(world, exp_mut):
        return False
    dev = arena.data.device
    cap = _cap(exp_mut, min(n, N_CAP))
    if not _blob_ok(world, L, lambda: [_m().gp_blob_bytes(0, n, cap, _token_p(world), L, D_CAP, K_CAP, 0)]):
        return False
    b = _begin(world, "mut")
    _room(world, cap * _r16(L + K_CAP))
    k = _kin_desc(world, dev)
    nbytes = _m().gp_blob_bytes(0, n, cap, k.P, L, D_CAP, K_CAP, 0)
    blob = _blob(world, "mut", nbytes, dev)
    seed, call = _rng()
    slot = _m().gp_mutate(_arena_desc(world, b), _gen_desc(world, dev), k, float(p), float(p_indel), float(p_del),
                          seed, call, cap, K_CAP, D_CAP, _p(blob), _stream())
    lay = _m().gp_layout(0, n, cap, L, K_CAP, 0)
    sel = _view(blob, lay["sel"], n, torch.int64)
    _record(world, "mut", (p, p_indel, p_del), (seed, call), sel, slot, _Replay(blob, lay, cap, "sel"))
    return True


def recombinate_all(world, p: float, extra=None) -> bool:
    """Device-pipeline ``recombinate_cells()`` over all cells (one C++ call, gp.hip); False for the
    synchronous path.

    ``extra`` (strip-boundary recombination of a decomposed world, magicsoup_amd.parallel) adds
    ``extra.rows`` result rows after the local pairs' results: ``extra.apply(pair_count, out, out_w,
    out_len, out_rows, nres)`` (device pointers) writes them and the number of result rows to
    commit; they are committed after (so they override) the local results, in the same passes."""
    arena = world._genomes
    if world.n_cells < 2:
        return True
    if not enabled(world):
        return False
    n0, L0 = world.n_cells, int(arena.width)
    pc0 = _pair_cap(n0, 8 * p * _nt(world, n0, L0), extra) or min(n0, N_CAP) // 2
    _prepare_records(world, 2 * pc0 + (0 if extra is None else int(extra.rows)))
    n = world.n_cells
    if n < 2:
        return True
    L = int(arena.width)
    # upper bound: at most 4n neighbour pairs (each in one slot), each genome in at most 8 of them,
    # so at most 8 p times the total length (_nt); real counts are several times lower (occupancy),
    # so the bound may reach N_CAP:
    # a count above the pair capacity makes the call a no-op that reconcile replays (cap_skip)
    expected = 8 * p * _nt(world, n, L)
    if p * 2 * L > LAM_MAX or not _usable(world, expected, N_CAP):
        return False
    pcap = _pair_cap(n, expected, extra)  # pairs per call (two results each)
    if pcap is None:
        return False  # (the synchronous path commits the boundary results itself)
    xr0 = 0 if extra is None else int(extra.rows)
    if not _blob_ok(world, L, lambda: [_m().gp_blob_bytes(1, n, pcap, _token_p(world), L, D_CAP, K_CAP, xr0)]):
        return False
    dev = arena.data.device
    b = _begin(world, "rec")
    _room(world, (2 * pcap + (0 if extra is None else int(extra.rows))) * _r16(2 * L))
    sc = _scratch(world)
    keys, nbr = hip_ops.neighbor_slot_args(world)
    k = _kin_desc(world, dev)
    xr = 0 if extra is None else int(extra.rows)
    nbytes = _m().gp_blob_bytes(1, n, pcap, k.P, L, D_CAP, K_CAP, xr)
    blob = _blob(world, "rec", nbytes, dev)
    mark = sc.bufs.get("arena_mark")
    if mark is None or mark.numel() < arena.n:
        mark = sc.bufs["arena_mark"] = torch.zeros(max(arena.n, 1024) * 2, dtype=torch.int64, device=dev)
        sc.bufs["arena_gen"] = 0
    gen = sc.bufs["arena_gen"] = sc.bufs.get("arena_gen", 0) + 1
    nres = sc.get("gp_nres", 1, torch.int32, dev) if extra is not None else None
    seed, call = _rng()
    slot = _m().gp_recombine(_arena_desc(world, b), _gen_desc(world, dev), k, _p(keys), nbr, float(p), seed, call, pcap,
                             K_CAP, D_CAP, _p(mark), int(gen), extra, _p(nres), _p(blob), _stream())
    lay = _m().gp_layout(1, n, pcap, L, K_CAP, xr)
    nr = lay["nr"]
    _record(world, "rec", (p,), (seed, call), _view(blob, lay["cells"], nr, torch.int64), slot,
            _Replay(blob, lay, nr, "out_rows", mark=mark, gen=gen, direct=extra is not None))
    return True


class _Part:
    """One half of a merged ``evolve`` call, shaped like a :class:`_Pending` for :func:`_recommit`."""

    __slots__ = ("kind", "host", "replay")

    def __init__(self, kind, host, replay):
        self.kind, self.host, self.replay = kind, host, replay


class _PartHost:
    """Status words of one half of an ``evolve`` call: the parts slot holds {pairs, rec flags,
    mutated, mut flags}; presented as {count, flags, -, pairs} like a single call's slot."""

    __slots__ = ("parts", "kind")

    def __init__(self, parts: _StatusSlot, kind: str):
        self.parts, self.kind = parts, kind

    def __getitem__(self, i: int) -> int:
        if self.kind == "rec":
            return {0: 0, 1: self.parts[1], 2: 0, 3: self.parts[0]}[i]
        return {0: self.parts[2], 1: self.parts[3], 2: 0, 3: self.parts[2]}[i]


# why issues on a pending kill_divide's device count were declined (World._chain_bound; the caller
# then waits for the count): diagnostics for scripts/lab/call_order.py
BOUND_DECLINED = {"pending": 0, "caps": 0, "rows": 0, "pool": 0, "mem": 0}


def evolve(world, p_rec: float, p: float, p_indel: float, p_del: float, extra=None, arrivals=None,
           bound=None) -> bool:
    """``recombinate_cells(p=p_rec)`` followed by ``mutate_cells(p, p_indel, p_del)`` over all cells
    as ONE device chain (gp.hip gp_evolve): both are applied and committed in order, then the union
    of the changed cells is translated and built once -- the same genomes and parameters as the two
    calls one after the other, with one translation + build less on the side stream. ``extra``: a
    decomposed world's strip-boundary recombination (as for :func:`recombinate_all`). ``arrivals``:
    ``(first, count)``, cells whose parameters are built with the union (instead of by a
    :func:`rebuild_rows` chain of their own; at most ``N_CAP``). False if either call should take its
    own path (rates above the pipeline's usage rule, too few cells). ``bound``: (cell bound, device
    count words) -- issued while a kill_divide's counts are still on the device (World._chain_bound):
    sized for the bound, the kernels read the count; False (nothing issued) where the host state the
    issue touches would depend on the count."""
    arena = world._genomes
    n = int(bound[0]) if bound is not None else world.n_cells
    if n < 2 or not enabled(world):
        return False
    st = _state(world)
    if any(pd.kind in ("rec", "mut", "evo") for pd in st["pending"]):
        if bound is not None:
            BOUND_DECLINED["pending"] += 1
            return False
        reconcile(world)  # (before anything below reads the world state it may change)
        n = world.n_cells
        if n < 2:
            return False
    # records for the union's rebuilt cells (at most): made before anything below reads world state
    # (see _prepare_records); with chains issued on a device count enabled, the synchronous path
    # makes room for the next call as well: those cannot collect (World._chain_bound)
    from magicsoup_amd.models import world as world_mod

    # (the union's capacity at the current state sizes the reservation; re-read after it)
    L0 = int(arena.width)
    nt0 = _nt(world, n, L0)
    pc0 = _pair_cap(n, 8 * p_rec * nt0, extra) or min(n, N_CAP) // 2
    ucap_max = 2 * pc0 + _cap(p * nt0, min(n, N_CAP)) + (0 if extra is None else int(extra.rows)) + (
        0 if arrivals is None else int(arrivals[1]))
    kin = world.kinetics
    if bound is not None:
        if not kin._rows_available(ucap_max):
            BOUND_DECLINED["rows"] += 1
            return False
        _prepare_records(world, ucap_max, sync=False)
    else:
        room_next = world_mod._CHAIN_BOUND and n <= world_mod._CHAIN_BOUND_MAX
        _prepare_records(world, ucap_max, headroom=ucap_max if room_next else 0)
        n = world.n_cells
        if n < 2:
            return False
    L = int(arena.width)
    nt = _nt(world, n, L)
    exp_rec = 8 * p_rec * nt
    if (p_rec * 2 * L > LAM_MAX or p * L > LAM_MAX or not _usable(world, exp_rec, N_CAP)
            or not _usable(world, p * nt)):
        return False
    pcap = _pair_cap(n, exp_rec, extra)
    if pcap is None:
        return False  # (the caller issues the recombination on its own: see _pair_cap)
    st = _state(world)
    if any(pd.kind in ("rec", "mut", "evo") for pd in st["pending"]):
        if bound is not None:
            BOUND_DECLINED["pending"] += 1
            return False
        reconcile(world)
    dev = arena.data.device
    mcap = _cap(p * nt, min(n, N_CAP))
    kin = world.kinetics
    arr0, narr = (0, 0) if arrivals is None else (int(arrivals[0]), int(arrivals[1]))
    fresh = not st["pending"]
    xr = 0 if extra is None else int(extra.rows)
    room = (2 * pcap + xr) * _r16(2 * L) + mcap * _r16(L + K_CAP)
    tp = _token_p(world)
    if not _blob_ok(world, L, lambda: [_m().gp_blob_bytes(1, n, pcap, tp, L, D_CAP, K_CAP, xr),
                                       _m().gp_blob_bytes(0, n, mcap, tp, L, D_CAP, K_CAP, 0),
                                       _m().gp_evolve_union_bytes(2 * pcap + xr + mcap + narr, tp, D_CAP, L)]):
        if bound is not None:
            BOUND_DECLINED["mem"] += 1
        return False
    if bound is not None:
        # nothing here may wait for the count: the selections must fit the append + sort paths (the
        # count + selection passes size their grids by the count), the fresh rows must exist without
        # a recycling (it scans the live cells' row map) and the pool must have room without a
        # collection (it moves the live cells' genomes)
        sc_cap = int(_m().sel_sort_cap())
        if extra is not None or narr or max(pcap, mcap, 2 * pcap) > sc_cap:
            BOUND_DECLINED["caps"] += 1
            return False
        if arena.top_ub + room > arena.pool_cap:
            BOUND_DECLINED["pool"] += 1
            return False
    _room(world, room)
    br, bm, bu = _bufs(world, "rec"), _bufs(world, "mut"), _bufs(world, "evo")
    ar, am, au = _arena_desc(world, br), _arena_desc(world, bm), _arena_desc(world, bu)
    nd = (0, 0)
    if bound is not None:
        ar.n = am.n = au.n = n  # (grids and scratch for the bound; the kernels read the count)
        nd = (int(bound[1]), int(bound[2]))
    sc = hip_ops._scratch(world)
    keys, nbr = hip_ops.neighbor_slot_args(world, bound)
    k = _kin_desc(world, dev)
    blob_r = _blob(world, "rec", _m().gp_blob_bytes(1, n, pcap, k.P, L, D_CAP, K_CAP, xr), dev)
    blob_m = _blob(world, "mut", _m().gp_blob_bytes(0, n, mcap, k.P, L, D_CAP, K_CAP, 0), dev)
    nres = sc.get("gp_nres", 1, torch.int32, dev) if extra is not None else None
    ucap = 2 * pcap + xr + mcap + narr
    blob_u = _blob(world, "evo", _m().gp_evolve_union_bytes(ucap, k.P, D_CAP, L), dev)
    mark = sc.bufs.get("arena_mark")
    na = max(arena.n, n)
    if mark is None or mark.numel() < na:
        mark = sc.bufs["arena_mark"] = torch.zeros(max(na, 1024) * 2, dtype=torch.int64, device=dev)
        sc.bufs["arena_gen"] = 0
    gen = sc.bufs["arena_gen"] = sc.bufs.get("arena_gen", 0) + 1
    rng_r, rng_m = _rng(), _rng()
    mirror = _top_mirror(world)
    _m().mapped_i64_write(mirror[0], -1)
    st["mirror_mark"] = (arena.collects, arena.inc_total, mirror[0])
    slot_u, slot_p = _m().gp_evolve(ar, am, au, _gen_desc(world, dev), k, _p(keys), nbr, float(p_rec), rng_r[0],
                                    rng_r[1], pcap, float(p), float(p_indel), float(p_del), rng_m[0], rng_m[1], mcap,
                                    K_CAP, D_CAP, _p(mark), int(gen), _p(blob_r), _p(blob_m), _p(blob_u), fresh,
                                    -1, extra, _p(nres), arr0, narr, nd[0], nd[1], mirror[1],
                                    _stream())
    lay_r = _m().gp_layout(1, n, pcap, L, K_CAP, xr)
    lay_m = _m().gp_layout(0, n, mcap, L, K_CAP, 0)
    parts = _StatusSlot(slot_p)
    replay = {
        "rec": _Part("rec", _PartHost(parts, "rec"), _Replay(blob_r, lay_r, lay_r["nr"], "out_rows", mark=mark, gen=gen,
                                                              direct=extra is not None)),
        "mut": _Part("mut", _PartHost(parts, "mut"), _Replay(blob_m, lay_m, mcap, "sel")),
    }
    cells = _view(blob_u, 0, ucap, torch.int64)
    _record(world, "evo", (p_rec, p, p_indel, p_del), (rng_r, rng_m), cells, slot_u, replay)
    return True


def _rebuild_set(pd):
    """Cells of a resolved call whose device-built parameters need the synchronous rebuild: all of
    the call's cells when the records outgrew the storage or the overflow list, the listed ones when
    only some proteomes outgrew the speculative token layout (gp.hip gp_check_assign_kernel), else
    None."""
    flags = int(pd.host[1])
    if flags & (_F_TRANSLATE | _F_ROWS):
        return pd.cells[: int(pd.host[0])]
    if flags & _F_PARTIAL:
        bad = _m().status_bad_read(pd.host._slot)
        return torch.tensor(bad, dtype=torch.long, device=pd.cells.device)
    return None


def _resolve_evo(world, pd) -> bool:
    """Reconcile a merged ``evolve`` call: each half like a call of its own (replay when skipped,
    re-commit when a result outgrew the arena), then the union's translation flags."""
    p_rec, p, p_indel, p_del = pd.args
    rng_r, rng_m = pd.rng
    rec, mut = pd.replay["rec"], pd.replay["mut"]
    fr, fm = int(rec.host[1]), int(mut.host[1])
    if (fr | fm) & _F_CAPACITY:
        raise RuntimeError("genome pipeline capacity exceeded (rates far above the pipeline's usage rule)")
    changed = []
    rebuilt = False
    if fr & _F_SKIPPED and rec.replay.direct:
        # (the recombination is the first call of a fresh chain: nothing before it can break the
        # chain, and a replay of the local pairs alone would lose the strip-boundary results)
        raise RuntimeError("genome pipeline: merged chain with boundary recombination was skipped")
    if fr & (_F_SKIPPED | _F_WIDTH):
        rebuilt = True
        if fr & _F_SKIPPED:
            changed.append(hip_ops.recombinate_all(world, p_rec, rng=rng_r))
        else:
            changed.append(_recommit(world, rec))
    if fm & _F_SKIPPED:  # (also whenever the recombination overflowed: the chain stopped there)
        rebuilt = True
        changed.append(hip_ops.point_mutations(world, None, p, p_indel, p_del, rng=rng_m))
    elif fm & _F_WIDTH:
        rebuilt = True
        changed.append(_recommit(world, mut))
    part = _rebuild_set(pd)
    if part is not None:
        rebuilt = True
        changed.append(part)
    changed = [c for c in changed if c.numel()]
    if changed:
        world._update_params_rows(torch.unique(torch.cat([c.to(torch.long) for c in changed])))
    return rebuilt


def rebuild_rows(world, rows: torch.Tensor) -> bool:
    """Translate and build parameters of the cells ``rows`` (e.g. spawned cells, or cells that
    arrived from another rank) into fresh parameter rows without a synchronisation (one C++ call,
    gp.hip gp_rebuild); resolved by :func:`reconcile` like the other pipeline calls. False if the
    caller should take the synchronous path."""
    k = int(rows.numel())
    if k == 0:
        return True
    if not enabled(world) or k > 8 * N_CAP or world.kinetics._P() == 0:
        return False  # (no protein slots yet: the synchronous path sizes the storage)
    Lw = int(world._genomes.width)
    if not _blob_ok(world, Lw, lambda: [_m().gp_blob_bytes(2, k, k, _token_p(world), Lw, D_CAP, 0, 0)]):
        return False
    if k > N_CAP:
        reconcile(world)  # (a large batch, e.g. a big top-up: a fresh chain)
    _prepare_records(world, k)
    b = _begin(world, "imm")
    dcnt = b["cnt"]
    dcnt[:1].fill_(k)
    cells = rows.to(torch.int64).contiguous()
    dev = cells.device
    kd = _kin_desc(world, dev)
    blob = _blob(world, "imm", _m().gp_blob_bytes(2, k, k, kd.P, int(world._genomes.width), D_CAP, 0, 0), dev)
    slot = _m().gp_rebuild(_arena_desc(world, b), _gen_desc(world, dev), kd, _p(cells), _p(dcnt), k, D_CAP,
                           _p(blob), _stream())
    _record(world, "imm", (), None, cells, slot, None)
    return True


def _recommit(world, pd: _Pending) -> torch.Tensor:
    """Commit a call's results after widening the arena to the longest one; returns the cells."""
    arena = world._genomes
    r = pd.replay
    if pd.kind == "mut":
        n_res = int(pd.host[0])
    else:  # recombination: 2 rows per pair, or the counted result rows (with strip-boundary results)
        n_res = int(pd.host[3]) if r.direct else 2 * int(pd.host[3])
    if n_res == 0:
        return torch.zeros(0, dtype=torch.long, device=arena.data.device)
    rows_all, out, out_w, out_len_all = r.views()
    out_len = out_len_all[:n_res]
    need = int(out_len.max().item())
    if need > arena.width:
        arena.reserve(arena.n, need)  # (the pool's length bound: nothing moves)
    rows = rows_all[:n_res]
    _room(world, n_res * _r16(min(out_w, arena.width)))
    _m().arena_scatter(n_res, 0, 1, _p(rows), _p(out), out_w, _p(out_len), _p(arena.data), _p(arena.off),
                       _p(arena.top), arena.pool_cap, int(arena.width), _p(arena.lens), _p(r.mark), int(r.gen), 0, 0, 0,
                       _stream())
    arena.version += 1
    return torch.unique(rows)


def reconcile(world) -> None:
    """Resolve pending device-pipeline calls, in issue order: adopt the device row counter,
    commit results that did not fit the arena (then replay the calls that were skipped because of
    it), and rebuild flagged cells on the synchronous path. An enzymatic_activity that was issued
    on top of the pending calls (World: speculative activity, single-process worlds) is undone and
    run again if any of this changed parameters."""
    d = world.__dict__
    st = d.get("_gp_state")
    spec = d.pop("_spec", None)
    pend = st["pending"] if st else []
    if not pend:
        return
    st["pending"] = []
    redo = _resolve(world, pend)
    if not redo or spec is None:
        return
    from magicsoup_amd.ops import world_ops

    hip_ops.restore_cell_state(world, spec)
    world_ops.enzymatic_activity(world)


def _top_mirror(world) -> tuple[int, int]:
    """(host, device) address of the mapped int64 into which a merged chain writes the pool's bump
    counter after its last allocation (gp.hip gp_union_kernel)."""
    c = _cache(world)
    mm = c.get("top_mirror")
    if mm is None:
        mm = c["top_mirror"] = _m().mapped_i64()
    return mm


def _tighten_pool_bound(world) -> None:
    """With every issued chain complete: the host bound of the pool counter becomes the last merged
    chain's mirrored counter plus what was reserved since that chain's issue (instead of the sum of
    every call's worst case since the last read-back). Keeps the device-count issue
    (World._chain_bound) from being declined for pool room that was reserved but never used."""
    mm = _state(world).get("mirror_mark")
    arena = world._genomes
    if mm is None or mm[0] != arena.collects or mm[2] != _top_mirror(world)[0]:
        return
    v = int(_m().mapped_i64_read(mm[2]))
    if v >= 0:
        arena.top_ub = min(arena.top_ub, v + arena.inc_total - mm[1])


def _resolve(world, pend: list) -> bool:
    """True if any genome or parameter was changed on the host."""
    rebuilt = False
    kin = world.kinetics
    pend[-1].event.synchronize()
    _tighten_pool_bound(world)
    # (the device record counter after the chain's last build: the host bound tightens to it plus
    # what was reserved since the chain started)
    kin._adopt_rtop(int(pend[-1].host[2]), _state(world).get("res_mark"))
    for pd in pend:
        if pd.kind == "evo":
            rebuilt |= _resolve_evo(world, pd)
            continue
        flags = int(pd.host[1])
        if flags & _F_CAPACITY:
            raise RuntimeError("genome pipeline capacity exceeded (rates far above the pipeline's usage rule)")
        if flags & _F_SKIPPED:
            # a predecessor's result did not fit the arena: run this call now, same RNG stream
            rebuilt = True
            if pd.kind == "mut":
                changed = hip_ops.point_mutations(world, None, *pd.args, rng=pd.rng)
            else:
                changed = hip_ops.recombinate_all(world, *pd.args, rng=pd.rng)
            if changed.numel():
                world._update_params_rows(changed)
            continue
        if flags & _F_WIDTH:
            rebuilt = True
            cells = _recommit(world, pd)
            if cells.numel():
                world._update_params_rows(cells)
            continue
        cells = _rebuild_set(pd)
        if cells is not None:
            # parameters are a pure function of the current genome: rebuild on the synchronous path
            rebuilt = True
            if cells.numel():
                world._update_params_rows(torch.unique(cells))
    return rebuilt
