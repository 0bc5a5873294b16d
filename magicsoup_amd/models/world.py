"""The simulation world: cells on a toroidal map, molecules on a per-species map.

Public API and semantics follow the reference ``python/magicsoup/world.py`` (class ``World``,
``world.py:36-1004``): the same constructor arguments, methods, return values and public state
(``cell_genomes``, ``cell_labels``, ``cell_map``, ``cell_positions``, ``cell_lifetimes``,
``cell_divisions``, ``cell_molecules``, ``molecule_map``, ``n_cells``, ``genetics``, ``kinetics``,
``chemistry``) and the same ``save_state`` / ``load_state`` file format.

MI355X-first design:

* every per-cell array lives in a capacity-managed device buffer; the public tensors are views,
  so spawning / dividing appends without re-copying the population (reference ``_expand_c`` +
  ``torch.cat`` on every call, ``world.py:986-989``);
* genomes and labels live in device byte arenas (:mod:`magicsoup_amd.models.strings`); the public
  ``cell_genomes`` / ``cell_labels`` are lazy list views;
* translation, parameter build, the kinetics integrator, diffusion / permeation / degradation,
  placement, neighbour search, mutation and recombination run as gfx950 HIP kernels
  (:mod:`magicsoup_amd.ops.hip_ops`) for GPU worlds and in the OpenMP host core for CPU worlds;
* API calls accept index lists (reference) or device index tensors (no host round trip), and
  ``*_t`` variants return tensors instead of Python lists.
"""
from __future__ import annotations

import functools
import gc
import math
import os
import pickle
import random
from pathlib import Path
from typing import Any, Sequence

import numpy as np
import torch

from magicsoup_amd.models.containers import Cell, Chemistry
from magicsoup_amd.models.genetics import Genetics
from magicsoup_amd.models.kinetics import Kinetics
from magicsoup_amd.models.strings import PoolArena, StringArena, StringColumn, pack_strings
from magicsoup_amd.ops import world_ops
from magicsoup_amd.utils.util import randstr
from magicsoup_amd.utils import profiling
from magicsoup_amd.utils.profiling import range_pop, range_push

_LABEL_LEN = 12
# ops that neither read genomes / parameters nor change cells or positions: pending device-pipeline
# genome updates (magicsoup_amd.ops.genome_pipeline) stay pending across them; every other op
# resolves them first
_PIPELINE_SAFE_OPS = frozenset({"mutate_cells", "recombinate_cells", "diffuse_molecules", "degrade_molecules",
                                "increment_cell_lifetimes"})
# ops that may run while the cell count of a division issued without a synchronisation
# (divide_cells_t(lazy=True)) is still on its way to the host: they queue genome chains or only touch
# the map / all capacity rows; diffuse_molecules adopts the count after its stencil launch
_COUNT_SAFE_OPS = frozenset({"mutate_cells", "recombinate_cells", "degrade_molecules", "diffuse_molecules"})
# (kill_divide's kill leaves rows past the survivors stale and children after them: until its counts
# are adopted only the ops above may run -- the degradation scales all capacity rows, which is
# harmless for stale ones)
_CHECK_ENV = os.environ.get("MS_CHECK_INVARIANTS") == "1"
_DEFER_ENV = os.environ.get("MS_DEFER_GENOME_OPS", "1")
# issue a queued recombinate + mutate pair on a pending kill_divide's device count (World._chain_bound)
# instead of waiting for the count on the host first: always (MS_CHAIN_BOUND=1), never (0), or by
# default for populations up to _CHAIN_BOUND_MAX cells. Small populations are host-bound and gain
# (1024^2 / 10k: +17 %); at 40-50k cells the bound-sized chain was 3-4 % slower in in-process A/Bs
# over 400 steps (scripts/lab/knob_ab.py, profiles/r5/devcount/).
_CHAIN_BOUND_ENV = os.environ.get("MS_CHAIN_BOUND", "auto")
_CHAIN_BOUND = _CHAIN_BOUND_ENV != "0"
_CHAIN_BOUND_MAX = 1 << 30 if _CHAIN_BOUND_ENV == "1" else 16384
# The genome chains flushed onto the side stream (World._flush_deferred) are joined into the compute
# stream at the next op that needs their results (the activity, or a read of genomes / parameters),
# not right after the flush: the molecule-only work in between (the lifetimes, the loop's masks)
# runs while the chains finish (single-process worlds; a strip of a decomposed world joins at once).


class _Deferred:
    """A queued all-cells genome operation (World._defer): the call, plus its kind ("rec" / "mut")
    and rates so that a recombination followed by a mutation can be issued as one device chain."""

    __slots__ = ("fn", "kind", "args")

    def __init__(self, fn, kind: str, args: tuple):
        self.fn, self.kind, self.args = fn, kind, args

    def __call__(self):
        return self.fn()


def _op(name: str):
    """Instrument a public World operation: roctx range (``MS_ROCTX=1``), per-op HIP-event timing
    (:meth:`World.enable_timings`) and invariant checks after the op (:meth:`World.set_debug_checks`
    or ``MS_CHECK_INVARIANTS=1``). Only the outermost op of a nested call is timed / checked; with
    nothing enabled the wrapper is one dict lookup."""

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(self, *args, **kwargs):
            d = self.__dict__
            if d.get("_count_pending") is not None and name not in _COUNT_SAFE_OPS:
                self._resolve_count()
            if d.get("_spec") is not None:
                self._reconcile()  # a speculative activity is confirmed (or redone) before anything else
            if (d.get("_gp_state") or d.get("_deferred")) and name not in _PIPELINE_SAFE_OPS:
                if name == "enzymatic_activity" and self._speculate():
                    self._flush_deferred()  # issue the queued chains; confirmed after the activity
                else:
                    self._reconcile()
            if d.get("_side_join") is not None and name not in _PIPELINE_SAFE_OPS:
                self._join_side()
            timer, check = d.get("_timer"), d.get("_debug_checks", _CHECK_ENV)
            if timer is None and not check and not profiling.roctx_enabled():
                return fn(self, *args, **kwargs)
            depth = d.get("_op_depth", 0)
            d["_op_depth"] = depth + 1
            range_push(name)
            try:
                if timer is not None and depth == 0:
                    with timer.phase(name):
                        out = fn(self, *args, **kwargs)
                else:
                    out = fn(self, *args, **kwargs)
                if check and depth == 0:
                    self.check_invariants(where=name)
                return out
            finally:
                range_pop()
                d["_op_depth"] = depth

        return wrapper

    return deco


def _diffusion_weights(rate: float) -> tuple[float, float]:
    """Stencil weights (neighbour a, centre b) for a diffusivity (reference world.py:948-971)."""
    rate = min(abs(rate), 1.0)
    if rate == 0.0:
        return 0.0, 1.0
    d = 1 / rate
    a = 1 / (d + 8)
    b = d * a
    b = b + 1.0 - (8 * a + b)
    return a, b


def _permeation_factor(rate: float) -> float:
    """Per-step exchange fraction for a permeability (reference world.py:935-946)."""
    rate = min(abs(rate), 1.0)
    if rate == 0.0:
        return 0.0
    return 1 / (1 / rate + 1)


class _Column:
    """A capacity-managed per-cell buffer exposed as a cached view of its first ``n`` rows.

    ``spare`` is a second buffer of the same capacity: an order-preserving compaction gathers the
    surviving rows into it and the two are swapped (no copy back)."""

    __slots__ = ("buf", "_view", "_n", "spare")

    def __init__(self, buf: torch.Tensor):
        self.buf = buf
        self._view: torch.Tensor | None = None
        self._n = -1
        self.spare: torch.Tensor | None = None

    def view(self, n: int) -> torch.Tensor:
        if self._view is None or self._n != n:
            self._view = self.buf if self.buf.size(0) == n else self.buf[:n]
            self._n = n
        return self._view

    def adopt(self, t: torch.Tensor, n: int) -> None:
        if t is self._view:
            return
        self.buf = t
        self._view = t
        self._n = n

    def reserve(self, n_old: int, n_new: int) -> None:
        if n_new <= self.buf.size(0):
            return
        cap = max(n_new, int(self.buf.size(0) * 1.5) + 64)
        nb = torch.zeros(cap, *self.buf.shape[1:], dtype=self.buf.dtype, device=self.buf.device)
        if n_old:
            nb[:n_old] = self.view(n_old)
        self.buf = nb
        self._view = None

    def spare_rows(self, k: int) -> torch.Tensor:
        sp = self.spare
        b = self.buf
        if sp is None or sp.size(0) < max(k, b.size(0)) or sp.shape[1:] != b.shape[1:] or sp.dtype != b.dtype:
            sp = self.spare = torch.empty(max(k, b.size(0)), *b.shape[1:], dtype=b.dtype, device=b.device)
        return sp[:k]

    def swap(self) -> None:
        self.buf, self.spare = self.spare, self.buf
        self._view = None


class World:
    """State of a simulation and the operations that advance it.

    Parameters:
        chemistry: Molecules and reactions of the simulation.
        map_size: Pixels per side of the square, toroidal map.
        abs_temp: Absolute temperature in K (scales reaction equilibria).
        mol_map_init: ``"randn"`` (|N(10, 1)|) or ``"zeros"`` initial molecule map.
        start_codons / stop_codons: CDS delimiters for the genetics.
        device: Torch device of all state (``"cuda"`` = the MI355X via ROCm). Falls back to CPU when
            no GPU is present, like the reference.
        batch_size: Accepted for API compatibility (the reference ignores it as well).
        seed: Optional seed of all native RNG streams (placement, mutation, recombination).
    """

    # domain-decomposition hooks of the op layer (set by magicsoup_amd.parallel.DistributedWorld)
    _exchange_map_halo = None
    _allreduce_flags = None
    _allreduce_totals = None

    def __init__(
        self,
        chemistry: Chemistry,
        map_size: int = 128,
        abs_temp: float = 310.0,
        mol_map_init: str = "randn",
        start_codons: tuple[str, ...] = ("TTG", "GTG", "ATG"),
        stop_codons: tuple[str, ...] = ("TGA", "TAG", "TAA"),
        device: str = "cpu",
        batch_size: int | None = None,
        seed: int | None = None,
        map_dtype: torch.dtype = torch.float32,
    ):
        if not torch.cuda.is_available():
            device = "cpu"
        self.device = device
        if map_dtype not in (torch.float32, torch.bfloat16, torch.float16):
            raise ValueError(f"map_dtype must be float32, bfloat16 or float16, got {map_dtype}")
        # reduced-precision map storage is a GPU-kernel feature; host kernels are fp32-only
        self.map_dtype = map_dtype if torch.device(device).type == "cuda" else torch.float32
        self.batch_size = batch_size
        self.map_size = map_size
        self.abs_temp = abs_temp
        self.chemistry = chemistry
        if seed is not None:
            world_ops.set_seed(seed, device)

        self.genetics = Genetics(start_codons=start_codons, stop_codons=stop_codons)
        self.kinetics = Kinetics(
            chemistry=chemistry,
            abs_temp=abs_temp,
            device=device,
            scalar_enc_size=max(self.genetics.one_codon_map.values()),
            vector_enc_size=max(self.genetics.two_codon_map.values()),
        )

        self._link_kinetics()

        self.n_molecules = len(chemistry.molecules)
        self._int_mol_idxs = list(range(self.n_molecules))
        self._ext_mol_idxs = list(range(self.n_molecules, 2 * self.n_molecules))
        self._mol_degrads = [math.exp(-math.log(2) / m.half_life) for m in chemistry.molecules]
        self._diffusion = [_diffusion_weights(m.diffusivity) for m in chemistry.molecules]
        self._permeation = [_permeation_factor(m.permeability) for m in chemistry.molecules]

        dev = torch.device(device)
        m = self.n_molecules
        self.n_cells = 0
        # GPU genomes: a ragged pool (per-cell offsets, shared by parents and children); CPU worlds
        # keep fixed-width rows on purpose: the OpenMP host core (csrc/host: translation, mutations,
        # recombination) runs one thread per genome over contiguous row-major bytes, a division
        # copies rows with memcpy, and the pool's reasons -- no device-side widening when one genome
        # grows, parents and children sharing bytes without a copy kernel, a device bump allocator --
        # do not apply to host memory, where a row widening is one realloc of a few MB. Both stores
        # expose the same StringColumn / rows_of interface, so every op is storage-agnostic.
        self._genomes = PoolArena(dev) if dev.type == "cuda" else StringArena(dev, width=64)
        self._labels = StringArena(dev, width=16)
        self._genome_col = StringColumn(self._genomes)
        self._label_col = StringColumn(self._labels)
        self._cols = {
            "cell_molecules": _Column(torch.zeros(0, m, dtype=torch.float32, device=dev)),
            "cell_positions": _Column(torch.zeros(0, 2, dtype=torch.int32, device=dev)),
            "cell_lifetimes": _Column(torch.zeros(0, dtype=torch.int32, device=dev)),
            "cell_divisions": _Column(torch.zeros(0, dtype=torch.int32, device=dev)),
        }
        self.__dict__["_pending_scale"] = None
        self.__dict__["_pending_corr"] = None
        self.cell_map = torch.zeros(*self._map_shape(), dtype=torch.bool, device=dev)
        self.molecule_map = self._get_molecule_map(n=m, size=map_size, init=mol_map_init)

    def _link_kinetics(self) -> None:
        """Let the kinetics object resolve pending device-pipeline genome updates before any host
        access to its parameters (magicsoup_amd.ops.genome_pipeline)."""
        import weakref

        self.kinetics.__dict__["_owner"] = weakref.ref(self)

    def _defer_genome_op(self) -> bool:
        """Whether an all-cells mutate / recombinate is queued instead of issued now.

        Their device-pipeline chains return nothing and touch only genomes and parameters, so the
        ops the reference loop runs next (degrade, diffuse, lifetimes: molecules only) commute with
        them exactly. Queuing the host-side issue until the diffusion stencil has been launched
        (diffuse_molecules flushes the queue after it) or the next op that reads genomes,
        parameters, cells or positions (that op flushes the queue first, in call order, before
        anything else) moves ~0.2 ms of launch work per step behind the stencil already running on
        the GPU. RNG draws happen at issue time; no op that draws can run before the flush. Off with
        ``MS_DEFER_GENOME_OPS=0`` and while per-op timings are enabled."""
        d = self.__dict__
        if _DEFER_ENV == "0" or d.get("_timer") is not None or not self._genomes.data.is_cuda:
            return False
        from magicsoup_amd.ops import genome_pipeline

        return genome_pipeline.enabled(self)

    def _speculate(self) -> bool:
        """Whether enzymatic_activity may run before the pending device-pipeline calls are confirmed.

        The host confirmation waits for the rebuild chains, which share the device with the
        diffusion stencil; issuing the activity first keeps the device busy meanwhile. The state
        the activity changes is saved first; the next access to molecules, or the next op,
        confirms the calls and -- only if one had to be redone on the host -- restores that state
        and runs the activity again with the corrected parameters. Single-process GPU worlds only: a
        decomposed world's activity is collective, so a redo would have to be agreed by all ranks
        (measured no faster than waiting for the chains, which its strips issue early anyway)."""
        d = self.__dict__
        return (_DEFER_ENV != "0" and d.get("_timer") is None and self._genomes.data.is_cuda
                and getattr(self, "_allreduce_flags", None) is None)

    def _defer(self, fn) -> None:
        d = self.__dict__
        q = d.setdefault("_deferred", [])
        if not q:
            from magicsoup_amd.ops.streams import NEvent

            d["_defer_event"] = NEvent().record()
        q.append(fn)

    def _evolve(self, rec: "_Deferred", mut: "_Deferred", bound=None) -> int:
        """Issue a queued recombinate_cells() + mutate_cells() pair as one device chain. Returns how
        many of the two calls were issued, in order (2: merged; 1: the recombination only, e.g. a
        decomposed world whose collective part has run; 0: neither -- the caller issues them).
        ``bound``: issue on the device count of a pending kill_divide (see :meth:`_chain_bound`)."""
        from magicsoup_amd.ops import genome_pipeline

        if bound is not None:
            return 2 if self._n_floor() >= 1 and genome_pipeline.evolve(self, rec.args[0], *mut.args, bound=bound) else 0
        return 2 if self.n_cells >= 2 and genome_pipeline.evolve(self, rec.args[0], *mut.args) else 0

    def _chain_bound(self, q: list):
        """(upper bound, device count words) for issuing the queued recombinate_cells() +
        mutate_cells() pair before a pending kill_divide's counts reach the host, or None.

        The flush used to wait for those counts (the chains are sized by the population) and issue the
        chain only then: ~0.27 ms of host wait, after which the chain's Python and launches put its
        first kernel ~60 us behind the division's last (profiles/r5/call_order.txt). Instead the chain
        is issued on the bound 2 n0 (a kill_divide at most doubles the population) with its kernels
        reading the count from the division's device counters (survivors + placed children), and it
        starts on the device the moment the division ends. Only a single-process GPU world, with
        nothing else pending and nothing of the host state the chain's issue needs depending on the
        count (no pipeline call to reconcile, no speculative activity, the parameter storage compact
        with rows to spare, the genome pool with room: genome_pipeline.evolve checks the last two)."""
        d = self.__dict__
        pend = d["_count_pending"]
        if not _CHAIN_BOUND or len(pend) < 4 or not isinstance(pend[1], tuple) or len(q) != 2:
            return None
        if int(pend[0]) > _CHAIN_BOUND_MAX:
            return None
        if getattr(q[0], "kind", None) != "rec" or getattr(q[1], "kind", None) != "mut":
            return None
        if "_n_pix_global" in d or d.get("_spec") is not None or not self._genomes.data.is_cuda:
            return None
        st = d.get("_gp_state")
        if st and st["pending"]:
            return None
        kd = self.kinetics.__dict__
        if kd.get("_slot") is None or not kd.get("_compact"):
            return None
        dc = pend[3]
        return (2 * int(pend[0]), dc.data_ptr(), dc.data_ptr() + 8)

    def _join_side(self) -> None:
        """The compute stream waits (device-side) for the genome chains issued so far."""
        d = self.__dict__
        ev = d.pop("_side_join", None)
        if ev is not None:
            ev.wait()  # (the current stream)
        # the tensors the chains were issued against may return to the allocator now: any later
        # compute-stream allocation is ordered after the wait above
        d.pop("_side_keep", None)

    def _storage_refs(self) -> list:
        """Every per-cell storage tensor a genome chain may read while it runs on the side stream
        (columns and spares, genome / label arenas, kinetics row storage, its spares, the cell ->
        row map and free list). Issuing a chain can replace some of them (storage growth, a row
        recycle, an arena widening); holding these references until the compute stream has joined
        the chains keeps a replaced block out of the caching allocator, which would otherwise hand
        it to a compute-stream allocation while a side-stream kernel still reads it."""
        refs: list = []
        for col in self._cols.values():
            refs.append(col.buf)
            refs.append(col.spare)
        for arena in (self._genomes, self._labels):
            refs.append(arena.data)
            refs.append(arena.lens)
            refs.append(arena.__dict__.get("_spare"))
            refs.append(arena.__dict__.get("off"))
        kd = self.kinetics.__dict__
        refs.extend(kd.get("_store_d", {}).values())
        refs.extend(kd.get("_spare", {}).values())
        for k in ("_slot_buf", "_slot_spare", "_free", "_zero_row_t", "_rtop"):
            refs.append(kd.get(k))
        return refs

    def _flush_deferred(self) -> None:
        """Issue the queued genome ops, in call order, on a side stream: their chains run next to
        the diffusion stencil still executing on the compute stream (disjoint state), and the compute
        stream waits for them (device-side) before anything that follows."""
        from magicsoup_amd.ops.hip_ops import _stream
        from magicsoup_amd.ops.streams import NEvent, join, on_stream

        d = self.__dict__
        q = d.get("_deferred")
        if not q:
            return
        bound = None
        if d.get("_count_pending") is not None:
            bound = self._chain_bound(q)
            if bound is None:
                self._resolve_count()  # (the chains are sized by the cell count)
        d["_deferred"] = []
        side = d.get("_side_stream")
        if side is None:
            # high priority: the short chain kernels are dispatched ahead of the stencil's waiting
            # workgroups (the next op's reconcile waits for the chains)
            side = d["_side_stream"] = torch.cuda.Stream(device=self._genomes.data.device, priority=-1)
        main = _stream()
        side_raw = side.cuda_stream
        # the chains depend on the state as of the first queued call (recorded then), not on the
        # molecule-only work issued since (e.g. the diffusion stencil they run next to)
        d.pop("_defer_event").wait(side_raw)
        d["_side_active"] = True  # (a decomposed world's exchanges use its side-stream communicator)
        lazy = "_n_pix_global" not in d  # (see the note at the top of this module)
        # (the queued closures hold compute-stream tensors the chains read, e.g. index lists)
        keep = [q, self._storage_refs()] if lazy else None
        try:
            with on_stream(side):
                i = 0
                while i < len(q):
                    # recombinate_cells() then mutate_cells(): one chain with one rebuild (gp_evolve)
                    if (i + 1 < len(q) and getattr(q[i], "kind", None) == "rec"
                            and getattr(q[i + 1], "kind", None) == "mut"):
                        done = self._evolve(q[i], q[i + 1], bound) if bound is not None else 0
                        if not done:
                            if bound is not None:
                                bound = None
                                self._resolve_count()
                            done = self._evolve(q[i], q[i + 1])
                        if done:
                            i += done
                            continue
                    if bound is not None:
                        bound = None
                        self._resolve_count()
                    q[i]()
                    i += 1
        finally:
            d["_side_active"] = False
            if lazy:
                # joined at the next op that needs the chains' results; what the chains read stays
                # referenced until then (see _storage_refs)
                prev = d.get("_side_keep")
                d["_side_keep"] = keep if prev is None else (prev, keep)
                d["_side_join"] = NEvent().record(side_raw)
            else:
                join(main, side_raw)

    def _reconcile(self) -> None:
        if self.__dict__.get("_count_pending") is not None:
            self._resolve_count()
        if self.__dict__.get("_deferred"):
            self._flush_deferred()
        self._join_side()
        if self.__dict__.get("_gp_state") or self.__dict__.get("_spec") is not None:
            from magicsoup_amd.ops import genome_pipeline

            genome_pipeline.reconcile(self)

    def _map_shape(self) -> tuple[int, int]:
        """(rows, cols) of this process's map (a strip with halo rows in magicsoup_amd.parallel)."""
        return self.map_size, self.map_size

    # ------------------------------------------------------------------ public state
    def __getattr__(self, name):  # only reached for attributes not found normally
        d = self.__dict__
        cols = d.get("_cols")
        if cols is not None and name in cols:
            if d.get("_spec") is not None or d.get("_count_pending") is not None:
                self._reconcile()
            return cols[name].view(d["n_cells"])
        if name == "molecule_map" and "_molmap" in d:
            if d.get("_spec") is not None:
                self._reconcile()
            if d.get("_pending_scale") is not None or d.get("_pending_corr") is not None:
                from magicsoup_amd.ops import hip_ops

                hip_ops.apply_pending(self)
            return d["_molmap"]
        if name == "cell_map" and "_cell_map" in d:
            return d["_cell_map"]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        cols = self.__dict__.get("_cols")
        if self.__dict__.get("_spec") is not None and (name == "molecule_map" or (cols is not None and name in cols)):
            # a speculative activity is confirmed (or redone) before the user's values replace the
            # state it changed: a later rollback must not overwrite them
            self._reconcile()
        if cols is not None and name in cols:
            t = torch.as_tensor(value, device=self.device)
            want = torch.float32 if name == "cell_molecules" else torch.int32
            t = t.to(want).contiguous() if (t.dtype != want or not t.is_contiguous()) else t
            cols[name].adopt(t, int(t.size(0)))
            return
        if name == "molecule_map":
            t = torch.as_tensor(value, device=self.device)
            want = self.__dict__.get("map_dtype", torch.float32)
            if t.dtype != want or not t.is_contiguous():
                t = t.to(want).contiguous()
            self.__dict__["_molmap"] = t
            self.__dict__["_pending_scale"] = None
            self.__dict__["_pending_corr"] = None
            return
        if name == "cell_map":
            self._set_cell_map(value)
            return
        if name == "cell_genomes":
            self._reconcile()
            self._set_strings(self._genomes, list(value))
            return
        if name == "cell_labels":
            self._set_strings(self._labels, list(value))
            return
        super().__setattr__(name, value)

    def _set_cell_map(self, value) -> None:
        """Keep the occupancy map in a 4-byte aligned, 4-byte padded buffer (the placement kernels
        claim pixels with 32-bit atomics); assigning copies into the existing buffer."""
        t = torch.as_tensor(value, device=self.device).to(torch.bool)
        cur = self.__dict__.get("_cell_map")
        if cur is not None and cur.shape == t.shape:
            if t.data_ptr() != cur.data_ptr():
                cur.copy_(t)
            return
        n = t.numel()
        buf = torch.zeros((n + 3) // 4 * 4 + 4, dtype=torch.bool, device=self.device)
        view = buf[:n].view(t.shape)
        view.copy_(t)
        self.__dict__["_cell_map"] = view

    @property
    def cell_genomes(self) -> StringColumn:
        """Genomes ordered by cell index (a lazy ``list[str]`` view of the device arena)."""
        self._reconcile()
        return self._genome_col

    @property
    def cell_labels(self) -> StringColumn:
        """Labels ordered by cell index (a lazy ``list[str]`` view)."""
        if self.__dict__.get("_count_pending") is not None:
            self._resolve_count()
        return self._label_col

    @property
    def n_cells(self) -> int:
        """Number of living cells (adopts a pending division count first, see :meth:`divide_cells_t`)."""
        d = self.__dict__
        if d.get("_count_pending") is not None:
            self._resolve_count()
        return d["n_cells"]

    @n_cells.setter
    def n_cells(self, n: int) -> None:
        self.__dict__["n_cells"] = n

    def _n_floor(self) -> int:
        """A lower bound of the cell count that never waits for the device (a pending division only
        adds cells)."""
        d = self.__dict__
        pend = d.get("_count_pending")
        return pend[0] if pend is not None else d["n_cells"]

    def _resolve_count(self) -> None:
        """Adopt the winner count of a division issued with ``lazy=True``: wait for the event
        recorded after its launches (not for work queued since, e.g. a diffusion stencil), read the
        count from its pinned status slot and adopt the grown population."""
        from magicsoup_amd.ops import hip_ops

        d = self.__dict__
        n0, slot, ev = d["_count_pending"][:3]
        # (only the division's work: not what was queued since, e.g. a diffusion stencil; with
        # communicators alive a peer failure raises instead of hanging)
        hip_ops.guarded_sync(ev)
        if isinstance(slot, tuple):  # kill_divide_t: survivors, then the winners appended after them
            n_k = int(hip_ops._m().status_read(slot[0])[0])
            k = int(hip_ops._m().status_read(slot[1])[0])
            d["_count_pending"] = None
            d["last_kill"] = (n0, n_k)
            hip_ops.check_placement()
            # (adopted whenever rows moved, not only when the count changed: a step that kills as
            # many cells as it divides still compacted the arenas, whose string caches are keyed on
            # their version)
            if n_k != n0 or k:
                self._adopt_count(n_k + k)
            return
        k = int(hip_ops._m().status_read(slot)[0])
        # (the pending entry stays until the count is read: a failure above leaves it for a retry
        # instead of a world whose device rows and host count disagree)
        d["_count_pending"] = None
        hip_ops.check_placement()
        if k:
            self._adopt_count(n0 + k)

    def _set_strings(self, arena: StringArena, strs: list[str]) -> None:
        arena.clear()
        arena.append_strings(strs)

    # ------------------------------------------------------------------ capacity helpers
    def reserve_cells(self, n: int, genome_len: int | None = None, proteins: int | None = None) -> None:
        """Allocate capacity for a population of ``n`` cells at once: per-cell columns, label and
        genome-pool bookkeeping, genome bytes (``genome_len`` nt per cell, 1 byte each, with the
        pool grows its own headroom) and -- once a first proteome has fixed the protein dimension -- the
        kinetics parameter rows, ``proteins`` slots wide (utils.memory.protein_slots: room for the
        longer proteomes recombination creates, so the storage never widens). Large worlds (utils.memory.plan: hundreds of GB) should be grown
        this way: batch-wise growth re-allocates each buffer 1.5x at a time with the old and the new
        copy alive together."""
        self._reconcile()
        self._reserve(n)
        self._genomes.reserve(n)
        self._labels.reserve(n)
        if genome_len and isinstance(self._genomes, PoolArena):
            self._genomes.ensure(max(0, n - self.n_cells) * ((int(genome_len) + 15) // 16 * 16))
        if self._genomes.data.is_cuda and self.n_cells and self.kinetics._P():
            # the GPU's compact parameter storage (packed words + Kmr) before the reservation: a
            # first large batch built the dense reference layout (2.5x the bytes per row)
            self.kinetics._packed_params()
            self.kinetics._enter_slot_mode()
            if proteins and proteins > self.kinetics._P():
                self.kinetics.increase_max_proteins(int(proteins))
        self.kinetics.reserve_cells(n)

    def _reserve(self, n_new: int) -> None:
        for col in self._cols.values():
            col.reserve(self.n_cells, n_new)

    def _grow(self, k: int, zero: bool = True, params: bool = True) -> None:
        """Append k cell rows to every per-cell array (world + kinetics unless ``params``);
        zero-initialised unless the caller overwrites them all."""
        n = self.n_cells
        self._reserve(n + k)
        if zero:
            for col in self._cols.values():
                col.buf[n : n + k] = 0
        self.n_cells = n + k
        if params:
            self.kinetics.increase_max_cells(by_n=k, zero=zero)

    def _clone_rows(self, src: torch.Tensor, dst: torch.Tensor) -> None:
        """Append copies of cells ``src`` as the new rows ``dst`` (= n_cells, n_cells + 1, ...):
        columns, genome / label arena rows and kinetics parameters."""
        k = int(src.numel())
        n0 = self.n_cells
        if not src.is_cuda:
            self._grow(k)
            self._genomes.append_rows_from(src)
            self._labels.append_rows_from(src)
            for name, col in self._cols.items():
                if name != "cell_positions":
                    col.buf[n0 : n0 + k] = col.buf[src]
            self.kinetics.copy_cell_params(from_idxs=src, to_idxs=dst)
            return
        from magicsoup_amd.ops import hip_ops

        # children share their parent's parameter rows until either is re-translated: the cell ->
        # row map is cloned in the same gather as the columns and arenas
        slot_pairs = self.kinetics.slot_clone_pairs(n0, k)
        self._grow(k, zero=False, params=False)
        n = self.n_cells
        pairs = [(col.view(n), col.view(n)) for name, col in self._cols.items() if name != "cell_positions"]
        pairs += self._genomes.clone_pairs(k) + self._labels.clone_pairs(k) + slot_pairs
        hip_ops.gather_rows(pairs, k, src_rows=src, dst_rows=dst)
        self.kinetics.append_shared(src, gathered=bool(slot_pairs))

    def _idx_tensor(self, idxs, unique: bool = True) -> torch.Tensor:
        """Cell indices as a long tensor on the world's device (ascending and duplicate-free when
        ``unique``; lists are deduplicated on the host, tensors with a membership mask)."""
        if isinstance(idxs, torch.Tensor):
            t = idxs.to(self.device)
            if t.dtype == torch.bool:
                if t.is_cuda:
                    from magicsoup_amd.ops import hip_ops

                    return hip_ops.select(t, "set")[0]
                return torch.nonzero(t).flatten()
            t = t.to(torch.long).flatten()
            if unique and t.numel() > 1:
                mask = torch.zeros(self.n_cells, dtype=torch.bool, device=self.device)
                mask[t] = True
                t = torch.nonzero(mask).flatten()
            return t
        lst = list(idxs)
        if unique:
            lst = sorted(set(lst))
        return torch.tensor(lst, dtype=torch.long, device=self.device)

    # ------------------------------------------------------------------ queries
    def get_cell(self, by_idx: int | None = None, by_position: tuple[int, int] | None = None) -> Cell:
        """A :class:`Cell` view of the cell at index ``by_idx`` or at pixel ``by_position``.

        Raises ``ValueError`` if no cell lives at ``by_position``.
        """
        self._reconcile()
        idx = -1
        if by_idx is not None:
            idx = by_idx
        if by_position is not None:
            pos = torch.tensor(by_position, dtype=torch.int32, device=self.device)
            hits = torch.argwhere((self.cell_positions == pos).all(dim=1)).flatten().tolist()
            if len(hits) == 0:
                raise ValueError(f"Cell at {by_position} not found")
            idx = hits[0]
        return Cell(
            world=self,
            idx=idx,
            genome=self.cell_genomes[idx],
            position=tuple(self.cell_positions[idx].tolist()),  # type: ignore[arg-type]
            label=self.cell_labels[idx],
            n_steps_alive=int(self.cell_lifetimes[idx].item()),
            n_divisions=int(self.cell_divisions[idx].item()),
        )

    def get_neighbors(self, cell_idxs: list[int], nghbr_idxs: list[int] | None = None) -> list[tuple[int, int]]:
        """Unique pairs ``(a, b)``, ``a < b``, of cells in each other's Moore neighbourhood.

        Each cell of ``cell_idxs`` pairs with neighbouring cells of ``nghbr_idxs`` (default:
        ``cell_idxs`` itself).
        """
        pairs = self.get_neighbors_t(cell_idxs, nghbr_idxs).cpu()
        # tens of thousands of new tuples: with the collector running, their allocation triggers
        # full collections over every tracked object of the process (~40 ms each at 24k pairs)
        paused = gc.isenabled()
        if paused:
            gc.disable()
        try:
            return list(zip(pairs[:, 0].tolist(), pairs[:, 1].tolist()))
        finally:
            if paused:
                gc.enable()

    @_op("get_neighbors")
    def get_neighbors_t(self, cell_idxs, nghbr_idxs=None) -> torch.Tensor:
        """Tensor form of :meth:`get_neighbors`: int32 (k, 2) on the world's device."""
        frm = self._idx_tensor(cell_idxs)
        if frm.numel() == 0:
            return torch.zeros(0, 2, dtype=torch.int32, device=self.device)
        to = frm if nghbr_idxs is None else self._idx_tensor(nghbr_idxs)
        if to.numel() == 0:
            return torch.zeros(0, 2, dtype=torch.int32, device=self.device)
        return world_ops.neighbors(self, frm, to)

    # ------------------------------------------------------------------ cell lifecycle
    @_op("spawn_cells")
    def spawn_cells(self, genomes) -> list[int]:
        """Place new cells with ``genomes`` on random free pixels.

        Each new cell takes half of its pixel's molecules, gets a random label, lifetime 0 and
        0 divisions. If there are fewer free pixels than genomes, a random subset is spawned.
        ``genomes`` is a ``list[str]`` or a packed ``(bytes (k, L) uint8, lengths (k,))`` tuple.

        Returns the indices of the new cells.
        """
        rows, lens = self._as_packed(genomes)
        k = int(rows.size(0))
        if k == 0:
            return []
        if rows.is_cuda:
            return self._spawn_gpu(rows, lens)
        pos = world_ops.free_positions(self, k)
        kp = int(pos.size(0))
        if kp == 0:
            return []
        if kp < k:
            keep = torch.randperm(k, device=rows.device)[:kp]
            rows, lens = rows[keep], lens[keep]
            k = kp
        n0 = self.n_cells
        self._grow(k)
        self._genomes.append_packed(rows, lens)
        self._labels.append_packed(*self._random_labels(k))
        new = torch.arange(n0, n0 + k, device=self.device)
        self._place_new(n0, pos)
        world_ops.pickup_molecules(self, new, pos)
        self._build_params_async(new)
        return list(range(n0, n0 + k))

    def _spawn_gpu(self, rows: torch.Tensor, lens: torch.Tensor) -> list[int]:
        """spawn_cells on the GPU without a host round trip: every cell occupies its own pixel, so
        the free pixels of the owned rows are known on the host; the claim / init kernel always finds
        one for each of at most that many cells, and the parameters are built by the device genome
        pipeline."""
        from magicsoup_amd.ops import hip_ops

        R, C, r_lo, r_hi, _ = world_ops.geom(self)
        n0 = self.n_cells
        free = (r_hi - r_lo) * C - n0
        k = int(rows.size(0))
        if free <= 0:
            return []
        if k > free:
            keep = torch.randperm(k, device=rows.device)[:free]
            rows, lens = rows[keep], lens[keep]
            k = free
        self._reserve(n0 + k)
        self._genomes.reserve(n0 + k, int(rows.size(1)))
        self._labels.reserve(n0 + k, _LABEL_LEN)
        hip_ops.spawn_issue(self, rows, lens, n0)
        self.n_cells = n0 + k
        for arena in (self._genomes, self._labels):
            arena.n = n0 + k
            arena.version += 1
        self.kinetics.increase_max_cells(by_n=k, zero=True)
        self._build_params_async(torch.arange(n0, n0 + k, device=self.device))
        return list(range(n0, n0 + k))

    @_op("add_cells")
    def add_cells(self, cells: list[Cell]) -> list[int]:
        """Place :class:`Cell` objects on random free pixels, keeping their genome, label,
        intracellular molecules, lifetime and divisions (no molecule pickup)."""
        k = len(cells)
        if k == 0:
            return []
        pos = world_ops.free_positions(self, k)
        kp = int(pos.size(0))
        if kp == 0:
            return []
        if kp < k:
            cells = list(cells)
            random.shuffle(cells)
            cells = cells[:kp]
            k = kp
        n0 = self.n_cells
        self._grow(k)
        self._genomes.append_strings([c.genome for c in cells])
        self._labels.append_strings([c.label for c in cells])
        new = torch.arange(n0, n0 + k, device=self.device)
        self._place_new(n0, pos)
        mols = torch.stack([torch.as_tensor(c.int_molecules) for c in cells]).to(self.device, torch.float32)
        self.cell_molecules[n0:] = mols
        self.cell_lifetimes[n0:] = torch.tensor([c.n_steps_alive for c in cells], dtype=torch.int32)
        self.cell_divisions[n0:] = torch.tensor([c.n_divisions for c in cells], dtype=torch.int32)
        self._update_params_rows(new)
        return list(range(n0, n0 + k))

    def divide_cells(self, cell_idxs) -> list[tuple[int, int]]:
        """Let cells divide into a random free pixel of their Moore neighbourhood.

        Children are appended at the end, inherit genome, proteome and label; molecules are split
        evenly; both descendants get ``divisions + 1`` and lifetime 0. Cells without a free
        neighbour do not divide. Returns ``(parent_idx, child_idx)`` pairs.
        """
        parents, children = self.divide_cells_t(cell_idxs)
        return list(zip(parents.tolist(), children.tolist()))

    @_op("divide_cells")
    def divide_cells_t(self, cell_idxs, lazy: bool = False) -> tuple[torch.Tensor, torch.Tensor] | None:
        """Tensor form of :meth:`divide_cells`: (parents, children) long tensors.

        ``lazy=True`` (a boolean GPU mask over all cells; the reference loop discards the pairs,
        ``performance/run_simulation.py:91``): returns None and does not wait for the division. The
        winner count travels to pinned memory and is adopted when the host next needs it -- reading
        ``n_cells`` or a cell attribute, or any operation other than the genome ops, degradation
        and diffusion, which are issued against the device state meanwhile (diffusion adopts it
        after launching its stencil, by when the division has long finished on the device)."""
        empty = torch.zeros(0, dtype=torch.long, device=self.device)
        if (isinstance(cell_idxs, torch.Tensor) and cell_idxs.dtype == torch.bool and cell_idxs.is_cuda
                and cell_idxs.numel() == self.n_cells and self.n_cells > 0):
            return self._divide_mask_gpu(cell_idxs, lazy=lazy)
        idxs = self._idx_tensor(cell_idxs)
        if idxs.numel() == 0:
            return empty, empty
        parents, child_pos = world_ops.divide_placement(self, idxs)
        k = int(parents.numel())
        if k == 0:
            return empty, empty
        n0 = self.n_cells
        children = torch.arange(n0, n0 + k, device=self.device)
        self._clone_rows(parents, children)
        if child_pos.is_cuda:
            # the placement kernels already claimed the pixels in cell_map
            self.cell_positions[n0 : n0 + k] = child_pos
        else:
            self._place(children, child_pos)
        world_ops.split_cells(self, parents, children)
        return parents, children

    def _commit_divisions_gpu(self, par: torch.Tensor, npos: torch.Tensor, k: int,
                              exporters: torch.Tensor | None = None) -> torch.Tensor:
        """Children of ``par[:k]`` at pixels ``npos[:k]`` (int32 (k, 2), already claimed) as rows
        n_cells..: one commit launch (positions, halved molecules, divisions, lifetimes; also the
        ``exporters`` -- parents whose child lives on another rank) and one gather of the genome /
        label / parameter-row entries. Returns the children's indices."""
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.hip_ops import _m, _p, _stream

        n0 = self.n_cells
        self._reserve(n0 + k)
        kin = self.kinetics
        kin._enter_slot_mode()
        kin._slot_reserve(n0 + k)
        g, lab = self._genomes, self._labels
        g.reserve(n0 + k)
        lab.reserve(n0 + k)
        par = par[:k].to(torch.int64).contiguous()
        npos = npos[:k].to(torch.int32).contiguous()
        ne = 0 if exporters is None else int(exporters.numel())
        exp = None if not ne else exporters.to(torch.int64).contiguous()
        cols = self._cols
        _m().divide_commit_list(k, _p(par), _p(npos), n0, ne, _p(exp), self.n_molecules,
                                _p(cols["cell_positions"].buf), _p(cols["cell_molecules"].buf),
                                _p(cols["cell_divisions"].buf), _p(cols["cell_lifetimes"].buf), _stream())
        if k:
            sb = kin.__dict__["_slot_buf"]
            # (children share their parent's genome: offsets and lengths only)
            pairs = [(g.off[:n0], g.off[n0 : n0 + k]), (g.lens[:n0], g.lens[n0 : n0 + k]),
                     (lab.data[:n0], lab.data[n0 : n0 + k], lab.lens), (lab.lens[:n0], lab.lens[n0 : n0 + k]),
                     (sb[:n0], sb[n0 : n0 + k])]
            hip_ops.gather_rows(pairs, k, src_rows=par)
            self.n_cells = n0 + k
            for arena in (g, lab):
                arena.n = n0 + k
                arena.version += 1
            kd = kin.__dict__
            kd["_slot"] = sb[: n0 + k]
            kd["_ncells"] += k
        return torch.arange(n0, n0 + k, device=self.device)

    def _divide_mask_gpu(self, mask: torch.Tensor, lazy: bool = False) -> tuple[torch.Tensor, torch.Tensor] | None:
        """Division over a GPU mask with one synchronisation at the very end: placement, winner
        compaction, the commit of the new rows and the genome / label / parameter-row clone are all
        issued against the device-side winner count (one native call, fast.hip fast_divide) into
        capacity reserved for the worst case (every cell divides); the host then only adopts the
        count."""
        from magicsoup_amd.ops import hip_ops

        n = self.n_cells
        fw = self._fast_world(2 * n)
        mask = mask.view(torch.uint8) if mask.dtype == torch.bool else mask.to(torch.uint8)
        seed, call = hip_ops._rng()
        slot = hip_ops._m().fast_divide(fw, n, mask.contiguous().data_ptr(), seed, call, hip_ops._stream())
        if lazy:
            from magicsoup_amd.ops.streams import NEvent

            self.__dict__["_count_pending"] = (n, slot, NEvent().record())
            return None
        k = hip_ops.wait_count(slot)
        hip_ops.check_placement()
        if k == 0:
            empty = torch.zeros(0, dtype=torch.long, device=self.device)
            return empty, empty
        self._adopt_count(n + k)
        # (the parents' scratch buffer is reused by the next division)
        par = self.__dict__["_fw_bufs"]["par"][:k].clone()
        return par, torch.arange(n, n + k, device=self.device)

    def _adopt_count(self, n: int) -> None:
        """A native operation left ``n`` valid rows in every per-cell buffer (columns, arenas, the
        kinetics cell -> row map): adopt the count on the host."""
        self.n_cells = n
        for arena in (self._genomes, self._labels):
            arena.n = n
            arena.version += 1
        kd = self.kinetics.__dict__
        kd["_slot"] = kd["_slot_buf"][:n]
        kd["_ncells"] = n

    def _fast_world(self, need: int):
        """The FastWorld descriptor of this world's per-cell buffers (csrc/hip/fast.hip) with room
        for ``need`` rows. Buffers are grown first if needed (1.5x); the descriptor is rebuilt
        whenever any of its buffers was reallocated (its key is their addresses), so it never
        points at freed memory."""
        d = self.__dict__
        kin = self.kinetics
        kin._enter_slot_mode()
        cols = self._cols
        g, lab = self._genomes, self._labels
        kd = kin.__dict__
        objs = d.get("_fw_objs")
        if objs is not None and need <= objs[0]:
            # the same buffer objects as at the last build (a reallocated, swapped or collected buffer
            # is always a new tensor object; holding the old ones keeps their addresses from being
            # reused meanwhile): the descriptor is current, without the ~20 address reads of the key
            cur = (g.data, g.off, g.lens, lab.data, lab.lens, kd["_slot_buf"], kd["_slot_spare"], d["_cell_map"],
                   *(c.buf for c in cols.values()))
            if len(cur) == len(objs) - 1 and all(a is b for a, b in zip(cur, objs[1:])):
                return d["_fw"]
        cap = min(min(int(c.buf.size(0)) for c in cols.values()), g.capacity, lab.capacity,
                  int(kd["_slot_buf"].numel()))
        if cap < need:
            target = max(need, int(cap * 1.5) + 64)
            self._reserve(target)
            g.reserve(target)
            lab.reserve(target)
            kin._slot_reserve(target)
            cap = min(min(int(c.buf.size(0)) for c in cols.values()), g.capacity, lab.capacity,
                      int(kd["_slot_buf"].numel()))
        fw = d.get("_fw")
        key = (cap, lab.width, g.data.data_ptr(), g.off.data_ptr(), g.lens.data_ptr(), g.pool_cap, lab.data.data_ptr(),
               lab.lens.data_ptr(), kd["_slot_buf"].data_ptr(), kd["_slot_spare"].data_ptr(),
               self.__dict__["_cell_map"].data_ptr(), *(c.buf.data_ptr() for c in cols.values()))
        objs = (cap, g.data, g.off, g.lens, lab.data, lab.lens, kd["_slot_buf"], kd["_slot_spare"], d["_cell_map"],
                *(c.buf for c in cols.values()))
        if fw is not None and d.get("_fw_key") == key:
            d["_fw_objs"] = objs
            return fw
        from magicsoup_amd.ops import hip_ops

        for c in cols.values():
            c.spare_rows(cap)
        g.compact_pairs(cap)  # (allocates the arenas' spares at their capacity and width)
        lab.compact_pairs(cap)
        dev = g.data.device
        R, C, r_lo, r_hi, wrap = world_ops.geom(self)
        claim = d.get("_claim_map")
        if claim is None or claim.numel() != R * C or claim.device != dev:
            claim = torch.full((R * C,), 0x7FFFFFFF, dtype=torch.int32, device=dev)
            d["_claim_map"] = claim
        bufs = {name: torch.empty(cap, dtype=dt, device=dev) for name, dt in (
            ("sel", torch.int64), ("pending", torch.uint8), ("cand", torch.int64), ("result", torch.int64),
            ("wins", torch.int64), ("par", torch.int64), ("dmask", torch.uint8))}
        bufs["dcount"] = torch.zeros(4, dtype=torch.int32, device=dev)
        fw = hip_ops._m().FastWorld()
        fw.R, fw.C, fw.r_lo, fw.r_hi, fw.wrap, fw.m, fw.cap = R, C, r_lo, r_hi, int(wrap), self.n_molecules, cap
        names = ("cell_molecules", "cell_positions", "cell_lifetimes", "cell_divisions")
        fw.mols, fw.pos, fw.life, fw.div = (cols[k].buf.data_ptr() for k in names)
        fw.mols_sp, fw.pos_sp, fw.life_sp, fw.div_sp = (cols[k].spare.data_ptr() for k in names)
        gs, ls = g.__dict__["_spare"], lab.__dict__["_spare"]
        fw.g_off, fw.g_lens, fw.g_off_sp, fw.g_lens_sp = (g.off.data_ptr(), g.lens.data_ptr(), gs[0].data_ptr(),
                                                          gs[1].data_ptr())
        fw.gpool = g.args()
        fw.l_data, fw.l_lens, fw.l_data_sp, fw.l_lens_sp = (lab.data.data_ptr(), lab.lens.data_ptr(),
                                                            ls[0].data_ptr(), ls[1].data_ptr())
        fw.l_width = int(lab.width)
        fw.slot, fw.slot_sp = kd["_slot_buf"].data_ptr(), kd["_slot_spare"].data_ptr()
        fw.cell_map = hip_ops._cell_map_bytes(self).data_ptr()
        fw.sel, fw.pending, fw.cand, fw.result, fw.wins, fw.par = (bufs[k].data_ptr() for k in (
            "sel", "pending", "cand", "result", "wins", "par"))
        fw.dcount, fw.dcount2 = bufs["dcount"].data_ptr(), bufs["dcount"].data_ptr() + 8
        fw.dmask = bufs["dmask"].data_ptr()
        fw.claim = claim.data_ptr()
        fw.rounds = hip_ops._PLACE_ROUNDS
        fw.finalize()
        d["_fw"], d["_fw_key"], d["_fw_bufs"], d["_fw_objs"] = fw, key, bufs, objs
        return fw

    @_op("update_cells")
    def update_cells(self, genome_idx_pairs: list[tuple[str, int]]):
        """Replace the genomes of existing cells and re-derive their proteomes."""
        k = len(genome_idx_pairs)
        if k == 0:
            return
        paused = gc.isenabled()  # (tens of thousands of short-lived containers: see get_neighbors)
        if paused:
            gc.disable()
        try:
            genomes, idxs = zip(*genome_idx_pairs)
            rows = torch.from_numpy(np.fromiter(idxs, dtype=np.int64, count=k))
            arr, lens = pack_strings(list(genomes))
        finally:
            if paused:
                gc.enable()
        self._genomes.set_rows(rows, torch.from_numpy(arr), torch.from_numpy(lens))
        self._update_params_rows(rows.to(self.device))

    @_op("kill_divide")
    def kill_divide_t(self, kill_mask: torch.Tensor, divide_mask: torch.Tensor) -> None:
        """``kill_cells(kill_mask)`` followed by ``divide_cells_t(divide_mask[~kill_mask], lazy=True)``
        in one call that never waits for the device: both masks are boolean over the current cells
        (the reference loop's kill and replicate steps, ``performance/run_simulation.py:80-92``, with
        the replicate mask taken before the kill -- the kill does not change a survivor's molecules,
        so it selects the same cells). On the GPU the survivors are compacted, the division mask with
        them, and the children appended after the device-side survivor count; both counts reach the
        host like a lazy division's (:meth:`divide_cells_t`). ``last_kill`` then holds the
        ``(cells before, survivors)`` of the last such call."""
        n = self.n_cells
        kill_mask = kill_mask.to(self.device, torch.bool)
        divide_mask = divide_mask.to(self.device, torch.bool)
        if kill_mask.numel() != n or divide_mask.numel() != n:
            raise ValueError(f"kill_divide_t: masks of {kill_mask.numel()} / {divide_mask.numel()} cells for {n}")
        if n == 0:
            if getattr(self, "_exchange_map_halo", None) is not None:  # (collective: see below)
                self.__dict__["last_kill"] = (0, 0)
                self.divide_cells_t(torch.zeros(0, dtype=torch.long, device=self.device))
            return
        if not kill_mask.is_cuda or getattr(self, "_exchange_map_halo", None) is not None:
            # CPU worlds, and a decomposed world's strips (their division is a collective protocol):
            # the two calls
            div = divide_mask[~kill_mask]
            self.kill_cells(kill_mask)
            self.__dict__["last_kill"] = (n, self.n_cells)
            if self.n_cells > 0:
                self.divide_cells_t(div, lazy=kill_mask.is_cuda)
            elif getattr(self, "_exchange_map_halo", None) is not None:
                # (the strip division is collective: an emptied strip still takes part)
                self.divide_cells_t(torch.zeros(0, dtype=torch.long, device=self.device))
            return
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.streams import NEvent

        fw = self._fast_world(2 * n)
        mm, corr = hip_ops.map_for_pixels(self)
        seed, call = hip_ops._rng()
        slots = hip_ops._m().fast_kill_divide(fw, n, kill_mask.view(torch.uint8).contiguous().data_ptr(),
                                              divide_mask.view(torch.uint8).contiguous().data_ptr(), mm.data_ptr(),
                                              hip_ops._mdt(mm), hip_ops._p(corr), seed, call, hip_ops._stream())
        # (+ the device counters {survivors, max, winners, max}: a genome chain may be issued on them
        # before the counts reach the host, see _chain_bound)
        self.__dict__["_count_pending"] = (n, tuple(slots), NEvent().record(), self.__dict__["_fw_bufs"]["dcount"])

    @_op("kill_divide")
    def kill_divide_where(self, molecule, kill_below: float, divide_above: float, divide_cost: float = 0.0,
                          kill_fraction: float = 0.0) -> None:
        """The reference loop's kill / replicate step as one call: cells whose ``molecule`` (index
        or name) is below ``kill_below`` die -- and, with ``kill_fraction`` > 0, each cell also dies
        with that probability (a chemostat dilution) --, surviving cells with more than
        ``divide_above`` of it pay ``divide_cost`` and divide (``performance/run_simulation.py:80-92``:
        kill below 1, divide above 5 at a cost of 4). Same semantics as building the two masks and
        calling :meth:`kill_divide_t`; on the GPU the masks, the payment, the kill and the division
        are one native call with no host synchronisation."""
        mol = self.chemistry.molname_2_idx[molecule] if isinstance(molecule, str) else int(molecule)
        if not 0 <= mol < self.n_molecules:
            raise ValueError(f"kill_divide_where: molecule index {mol} out of range")
        n = self.n_cells
        strip = getattr(self, "_exchange_map_halo", None) is not None
        if n == 0:
            if strip:  # (the strip division is collective: an empty strip still takes part)
                self.__dict__["last_kill"] = (0, 0)
                self.divide_cells_t(torch.zeros(0, dtype=torch.long, device=self.device))
            return
        if self._genomes.data.is_cuda and strip:
            native = getattr(self, "_kill_divide_native", None)
            if native is not None and native(n, mol, kill_below, divide_above, divide_cost, kill_fraction):
                return
            # a decomposed world's strip: native masks and kill (its one synchronisation), the
            # division mask compacted with the survivors on the device, then the strip's lazy
            # division protocol
            from magicsoup_amd.ops import hip_ops

            fw = self._fast_world(2 * n)
            bufs = self.__dict__["_fw_bufs"]
            cap = int(bufs["sel"].numel())
            if bufs.get("kmask") is None or bufs["kmask"].numel() < cap:
                bufs["kmask"] = torch.empty(cap, dtype=torch.uint8, device=self._genomes.data.device)
                bufs["dvmask"] = torch.empty_like(bufs["kmask"])
                bufs["dvmask2"] = torch.empty_like(bufs["kmask"])
            seed, call = hip_ops._rng() if kill_fraction > 0.0 else (0, 0)  # (no draws: no stream used)
            m_ = hip_ops._m()
            m_.fast_threshold_masks(fw, n, mol, float(kill_below), float(divide_above), float(divide_cost),
                                    float(kill_fraction), seed ^ 0x6A09E667F3BCC909, call, bufs["kmask"].data_ptr(),
                                    bufs["dvmask"].data_ptr(), hip_ops._stream())
            self.kill_cells(bufs["kmask"][:n].view(torch.bool))
            n_after = self.n_cells
            self.__dict__["last_kill"] = (n, n_after)
            if n_after > 0:
                fw = self._fast_world(n_after)  # (the kill's survivor indices are in this descriptor's sel)
                m_.fast_compact_mask(fw, n, bufs["dvmask"].data_ptr(), bufs["dvmask2"].data_ptr(), hip_ops._stream())
                self.divide_cells_t(bufs["dvmask2"][:n_after].view(torch.bool), lazy=True)
            else:
                self.divide_cells_t(torch.zeros(0, dtype=torch.long, device=self.device))
            return
        if not self._genomes.data.is_cuda:
            a = self.cell_molecules[:, mol]
            kill = a < kill_below
            if kill_fraction > 0.0:
                kill |= torch.rand(n, device=a.device) < kill_fraction
            div = (a > divide_above) & ~kill
            a -= divide_cost * div
            self.kill_divide_t(kill, div)
            return
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.streams import NEvent

        fw = self._fast_world(2 * n)
        mm, corr = hip_ops.map_for_pixels(self)
        bufs = self.__dict__["_fw_bufs"]
        kill = bufs.get("kmask")
        if kill is None or kill.numel() < int(bufs["sel"].numel()):
            kill = bufs["kmask"] = torch.empty(int(bufs["sel"].numel()), dtype=torch.uint8, device=mm.device)
            bufs["dvmask"] = torch.empty_like(kill)
        seed, call = hip_ops._rng()  # (the dilution draws use a key of their own on the same call)
        slots = hip_ops._m().fast_kill_divide_where(
            fw, n, mol, float(kill_below), float(divide_above), float(divide_cost), float(kill_fraction),
            seed ^ 0x6A09E667F3BCC909, call,
            kill.data_ptr(), bufs["dvmask"].data_ptr(), mm.data_ptr(), hip_ops._mdt(mm), hip_ops._p(corr), seed, call,
            hip_ops._stream())
        self.__dict__["_count_pending"] = (n, tuple(slots), NEvent().record(), bufs["dcount"])

    @_op("kill_cells")
    def kill_cells(self, cell_idxs=None):
        """Remove cells; their molecules spill onto their pixel. Remaining cells keep their order
        (indices after a removed cell shift down)."""
        n = self.n_cells
        if n == 0:
            return
        if cell_idxs is None:
            dead = torch.ones(n, dtype=torch.bool, device=self.device)
        elif isinstance(cell_idxs, torch.Tensor) and cell_idxs.dtype == torch.bool:
            dead = cell_idxs.to(self.device)
        else:
            t = cell_idxs if isinstance(cell_idxs, torch.Tensor) else torch.tensor(list(cell_idxs), dtype=torch.long)
            dead = torch.zeros(n, dtype=torch.bool, device=self.device)
            if t.numel() == 0:
                return
            dead.index_fill_(0, t.to(self.device, torch.long), True)  # duplicates are harmless
        if dead.is_cuda:
            from magicsoup_amd.ops import hip_ops

            # spill, survivor selection and the order-preserving compaction of every per-cell
            # buffer (into the spares and back) in one native call, launched against the
            # device-side survivor count before the one stream sync that brings it to the host
            fw = self._fast_world(n)
            mm, corr = hip_ops.map_for_pixels(self)
            mask = dead.view(torch.uint8) if dead.dtype == torch.bool else dead.to(torch.uint8)
            slot = hip_ops._m().fast_kill(fw, n, mask.contiguous().data_ptr(), mm.data_ptr(), hip_ops._mdt(mm),
                                          hip_ops._p(corr), True, hip_ops._stream())
            n_new = hip_ops.wait_count(slot)
            if n_new != n:
                self._adopt_count(n_new)
            return
        world_ops.spill_and_free_mask(self, dead)
        keep = ~dead
        keep_idx = torch.nonzero(keep).flatten()
        if int(keep_idx.numel()) == n:
            return
        self._compact(keep_idx, keep)

    def _compact(self, keep_idx: torch.Tensor, keep: torch.Tensor | None, removed: torch.Tensor | None = None) -> None:
        n_new = int(keep_idx.numel())
        if keep_idx.is_cuda:
            # every per-cell array (columns, arenas, kinetics parameters) in one gather launch
            # into spare buffers, then swap
            from magicsoup_amd.ops import hip_ops

            n = self.n_cells
            pairs = [(col.view(n), col.spare_rows(n_new)) for col in self._cols.values()]
            pairs += self._genomes.compact_pairs(n_new) + self._labels.compact_pairs(n_new)
            hip_ops.gather_rows(pairs, n_new, src_rows=keep_idx)
            # kinetics parameters stay where they are; only the cell -> row map is compacted
            self.kinetics.remove_cell_params(keep=keep_idx, removed=removed)
            for col in self._cols.values():
                col.swap()
            self._genomes.commit_compact(n_new)
            self._labels.commit_compact(n_new)
            self.n_cells = n_new
            return
        for col in self._cols.values():
            v = col.view(self.n_cells)
            col.buf[:n_new] = v[keep_idx]
            col._view = None
        self.kinetics.remove_cell_params(keep=keep_idx)
        self._genomes.keep(keep_idx)
        self._labels.keep(keep_idx)
        self.n_cells = n_new

    @_op("move_cells")
    def move_cells(self, cell_idxs=None):
        """Move cells to a random free pixel of their Moore neighbourhood (if there is one)."""
        if cell_idxs is None:
            cell_idxs = torch.arange(self.n_cells, device=self.device)
        idxs = self._idx_tensor(cell_idxs)
        if idxs.numel() == 0:
            return
        moved, new_pos = world_ops.move_placement(self, idxs)
        if moved.numel() == 0:
            return
        old = self.cell_positions[moved].long()
        self.cell_map[old[:, 0], old[:, 1]] = False
        self._place(moved, new_pos)

    @_op("reposition_cells")
    def reposition_cells(self, cell_idxs=None):
        """Move cells to random free pixels anywhere on the map."""
        if cell_idxs is None:
            cell_idxs = torch.arange(self.n_cells, device=self.device)
        idxs = self._idx_tensor(cell_idxs)
        if idxs.numel() == 0:
            return
        old = self.cell_positions[idxs].long()
        self.cell_map[old[:, 0], old[:, 1]] = False
        pos = world_ops.free_positions(self, int(idxs.numel()))
        if pos.is_cuda:
            self.cell_positions[idxs[: pos.size(0)]] = pos  # claimed by the kernel
        else:
            self._place(idxs[: pos.size(0)], pos)

    def _place(self, idxs: torch.Tensor, pos: torch.Tensor) -> None:
        pos = pos.to(self.device, torch.int32)
        self.cell_positions[idxs] = pos
        p = pos.long()
        self.cell_map[p[:, 0], p[:, 1]] = True

    def _place_new(self, n0: int, pos: torch.Tensor) -> None:
        """Positions of the new rows n0.. from world_ops.free_positions (on the GPU those pixels
        are already claimed in cell_map by the claim kernel)."""
        k = int(pos.size(0))
        if pos.is_cuda:
            self.cell_positions[n0 : n0 + k] = pos
        else:
            self._place(torch.arange(n0, n0 + k, device=self.device), pos)

    # ------------------------------------------------------------------ physics
    @_op("enzymatic_activity")
    def enzymatic_activity(self):
        """Let all proteins of all cells work for one time step (updates ``cell_molecules`` and
        the molecule map pixels under the cells)."""
        if self.n_cells == 0:
            return
        d = self.__dict__
        st = d.get("_gp_state")
        spec = save = None
        if st and st["pending"]:
            # speculative: issued on top of unconfirmed parameter rebuilds (see _speculate); the
            # fused activity snapshots what it changes in its own input pass
            from magicsoup_amd.ops import hip_ops

            if world_ops.fused_activity(self):
                spec = save = hip_ops.cell_state_buffer(self)
            else:
                spec = hip_ops.save_cell_state(self)
        world_ops.enzymatic_activity(self, save=save)
        if spec is not None:
            self.__dict__["_spec"] = spec

    @_op("diffuse_molecules")
    @torch.no_grad()
    def diffuse_molecules(self):
        """One step of diffusion over the molecule map, then membrane permeation."""
        world_ops.diffuse(self)
        if self.__dict__.get("_deferred"):
            # the stencil is queued: issue the deferred genome chains now, so that they start next to
            # it on the side stream instead of after the host has reached the next op (~0.1 ms later);
            # before the permeation's launch (molecules only: it commutes with the chains), which would
            # only delay them
            self._flush_deferred()
        if self.n_cells > 0:  # (adopts a pending division count: the stencil is queued already)
            world_ops.permeate(self)

    @_op("degrade_molecules")
    def degrade_molecules(self):
        """Decay molecules in the map and in cells by one time step (per-species half life)."""
        world_ops.degrade(self)

    @_op("increment_cell_lifetimes")
    def increment_cell_lifetimes(self):
        """Add 1 to every cell's lifetime."""
        lt = self.cell_lifetimes
        if lt.is_cuda and lt.numel() and lt.is_contiguous():
            from magicsoup_amd.ops import hip_ops

            hip_ops._m().add_i32(lt.numel(), lt.data_ptr(), 1, hip_ops._stream())  # (one native launch)
        else:
            self.cell_lifetimes += 1

    # ------------------------------------------------------------------ evolution
    @_op("mutate_cells")
    def mutate_cells(self, cell_idxs: list[int] | None = None, p: float = 1e-6, p_indel: float = 0.4, p_del: float = 0.66):
        """Point mutations (substitutions and indels) with per-bp rate ``p``; proteomes of mutated
        cells are re-derived."""
        if self._n_floor() == 0 and self.n_cells == 0:
            return
        if cell_idxs is None and self._defer_genome_op():
            self._defer(_Deferred(lambda: self._mutate_all(p, p_indel, p_del), "mut", (p, p_indel, p_del)))
            return
        if cell_idxs is None:
            return self._mutate_all(p, p_indel, p_del)
        self._reconcile()
        rows = self._idx_tensor(cell_idxs, unique=False)
        changed = world_ops.point_mutations(self, rows, p, p_indel, p_del)
        if changed.numel() > 0:
            self._update_params_rows(changed)

    def _mutate_all(self, p: float, p_indel: float, p_del: float) -> None:
        if self.n_cells == 0:
            return
        if self._genomes.data.is_cuda:
            from magicsoup_amd.ops import genome_pipeline

            if genome_pipeline.point_mutations(self, p, p_indel, p_del):
                return
        self._reconcile()
        rows = None
        changed = world_ops.point_mutations(self, rows, p, p_indel, p_del)
        if changed.numel() > 0:
            self._update_params_rows(changed)

    @_op("recombinate_cells")
    def recombinate_cells(self, cell_idxs: list[int] | None = None, p: float = 1e-7):
        """Recombine the genomes of neighbouring cells (strand breaks with per-bp rate ``p`` and
        random re-joining); both genomes of every recombined pair are replaced."""
        if self._n_floor() < 2 and self.n_cells < 2:
            return
        if cell_idxs is None and self._defer_genome_op():
            self._defer(_Deferred(lambda: self._recombinate_all(p), "rec", (p,)))
            return
        self._recombinate_all(p, cell_idxs)

    def _recombinate_all(self, p: float, cell_idxs=None) -> None:
        if self.n_cells < 2:
            return
        if cell_idxs is None and self._genomes.data.is_cuda:
            from magicsoup_amd.ops import genome_pipeline

            if genome_pipeline.recombinate_all(self, p):
                return
        self._reconcile()
        if cell_idxs is None and self._genomes.data.is_cuda:
            from magicsoup_amd.ops import hip_ops

            changed = hip_ops.recombinate_all(self, p)
        else:
            if cell_idxs is None:
                idxs = torch.arange(self.n_cells, device=self.device)
                pairs = world_ops.neighbors(self, idxs, idxs)
            else:
                pairs = self.get_neighbors_t(cell_idxs)
            if pairs.size(0) == 0:
                return
            changed = world_ops.recombinations(self, pairs, p)
        if changed.numel() > 0:
            self._update_params_rows(changed)

    # ------------------------------------------------------------------ params
    def _build_params_async(self, rows: torch.Tensor) -> None:
        """:meth:`_update_params_rows` through the device genome pipeline where it applies (GPU: no
        synchronisation; resolved at the next op like mutate / recombinate)."""
        if rows.is_cuda:
            from magicsoup_amd.ops import genome_pipeline

            if genome_pipeline.rebuild_rows(self, rows):
                return
        self._update_params_rows(rows)

    _PARAM_CHUNK = 1 << 18  # cells per translation + build: the token tensor is (k, P, D, 5) int32

    def _update_params_rows(self, rows: torch.Tensor) -> None:
        """Translate the genomes of ``rows`` and rebuild their kinetic parameters (in chunks: the
        token tensor of a multi-million-cell batch would take tens of GB)."""
        rows = rows.to(self.device, torch.long)
        if rows.numel() == 0:
            return
        if rows.numel() > self._PARAM_CHUNK:
            for c0 in range(0, int(rows.numel()), self._PARAM_CHUNK):
                self._update_params_rows(rows[c0 : c0 + self._PARAM_CHUNK])
            return
        tokens, nprots = world_ops.translate(self, rows)
        P = int(tokens.size(1))
        if P > self.kinetics._P():
            # a new longest proteome: grow with headroom on the GPU (1.5x) so that genomes growing
            # through recombination do not re-layout the parameter storage every few dozen steps
            # (padding proteins are inert: Vmax 0)
            from magicsoup_amd.models.kinetics import _MAX_PROTEINS

            grown = min(P + max(8, P // 2), max(P, _MAX_PROTEINS))  # (the headroom stops at the layout)
            self.kinetics.increase_max_proteins(grown if rows.is_cuda else P)
        # one build launch: rows without proteins are unset in the same pass
        self.kinetics.set_cell_params_tokens(rows, tokens, nprot=nprots)

    # ------------------------------------------------------------------ persistence
    def save(self, rundir: Path, name: str = "world.pkl"):
        """Pickle the whole world (chemistry, genetics, kinetics maps and state)."""
        rundir = Path(rundir)
        rundir.mkdir(parents=True, exist_ok=True)
        with open(rundir / name, "wb") as fh:
            pickle.dump(self, fh)

    @classmethod
    def from_file(cls, rundir: Path, name: str = "world.pkl", device: str | None = None) -> "World":
        """Restore a world written by :meth:`save` (optionally onto another device)."""
        from magicsoup_amd.utils.checkpoint import load_world_pickle

        return load_world_pickle(Path(rundir) / name, device=device)

    def __getstate__(self):
        self._reconcile()
        state = self.__dict__.copy()
        n = self.n_cells
        for k in ("_genome_col", "_label_col"):
            state.pop(k, None)
        state["_cols"] = {k: c.view(n).cpu().clone() for k, c in self._cols.items()}
        state["_genomes"] = self._genomes.to_strings()
        state["_labels"] = self._labels.to_strings()
        state["_molmap"] = self.molecule_map.cpu()
        state["_cell_map"] = self.cell_map.cpu()
        state["_pending_scale"] = None
        state["_pending_corr"] = None
        for k in ("_hip_scratch", "_idx_map", "_diff_w", "_perm_t", "_degrade_t", "_gp_state", "_deferred",
                  "_side_stream", "_defer_event", "_gp_cache", "_spec", "_halo_stream", "_side_join",
                  "_side_keep", "_fw", "_fw_key", "_fw_bufs", "_fw_objs"):
            state.pop(k, None)
        return state

    def __setstate__(self, state):
        if "_cols" not in state and "cell_molecules" in state:
            # a reference pickle (magicsoup.world.World, world.py:161-204): convert its layout
            from magicsoup_amd.utils.checkpoint import reference_world_state

            state = reference_world_state(state)
        dev = torch.device(state["device"] if torch.cuda.is_available() else "cpu")
        if dev.type == "cpu":
            state["device"] = "cpu"
        cols = state.pop("_cols")
        genomes = state.pop("_genomes")
        labels = state.pop("_labels")
        self.__dict__.update(state)
        self.__dict__["_cols"] = {k: _Column(v.to(dev)) for k, v in cols.items()}
        for c in self._cols.values():
            c.view(int(c.buf.size(0)))
        self.__dict__["_genomes"] = PoolArena(dev) if dev.type == "cuda" else StringArena(dev, width=64)
        self.__dict__["_labels"] = StringArena(dev, width=16)
        self._genomes.append_strings(genomes)
        self._labels.append_strings(labels)
        self.__dict__["_genome_col"] = StringColumn(self._genomes)
        self.__dict__["_label_col"] = StringColumn(self._labels)
        cmap = self.__dict__.pop("_cell_map")
        mdt = self.__dict__.get("map_dtype", torch.float32) if dev.type == "cuda" else torch.float32
        self.__dict__["map_dtype"] = mdt
        self.__dict__["_molmap"] = self.__dict__["_molmap"].to(dev, mdt).contiguous()
        self._set_cell_map(cmap.to(dev))
        self._link_kinetics()

    def to(self, device: str) -> "World":
        """Move all state of this world to ``device`` (returns ``self``)."""
        dev = torch.device(device)
        st = self.__getstate__()
        st["device"] = device
        self.__setstate__(st)
        kin = self.kinetics
        kin.device = device
        kin.__dict__.pop("_hip_scratch", None)
        kin._to_device(dev)
        for name, val in list(vars(kin).items()):
            if isinstance(val, torch.Tensor):
                kin.__dict__[name] = val.to(dev)
        for mp in (kin.km_map, kin.vmax_map, kin.sign_map, kin.hill_map, kin.reaction_map, kin.transport_map, kin.effector_map):
            for name, val in list(vars(mp).items()):
                if isinstance(val, torch.Tensor):
                    setattr(mp, name, val.to(dev))
        return self

    @_op("save_state")
    def save_state(self, statedir: Path):
        """Write the current state (tensors + ``cells.fasta``) in the reference's format, plus the
        random streams (``rng_state.pt``, ignored by the reference)."""
        self._reconcile()
        from magicsoup_amd.utils.checkpoint import save_state

        save_state(self, Path(statedir))

    @_op("load_state")
    def load_state(self, statedir: Path, ignore_cell_params: bool = False, restore_rng: bool = False):
        """Load a state written by :meth:`save_state` (re-translating genomes unless
        ``ignore_cell_params``). Restoring the random streams is opt-in: with ``restore_rng=True``
        and an ``rng_state.pt`` in the state (written by this package) the run continues exactly as
        an uninterrupted one would; by default (like the reference, which saves no RNG state) the
        streams continue from wherever this process's are."""
        self._reconcile()
        from magicsoup_amd.utils.checkpoint import load_state

        load_state(self, Path(statedir), ignore_cell_params=ignore_cell_params, restore_rng=restore_rng)

    # ------------------------------------------------------------------ internals
    def _as_packed(self, genomes) -> tuple[torch.Tensor, torch.Tensor]:
        if isinstance(genomes, tuple) and len(genomes) == 2 and isinstance(genomes[0], torch.Tensor):
            rows, lens = genomes
            return rows.to(self.device, torch.uint8), lens.to(self.device, torch.int32)
        genomes = list(genomes)
        arr, lens = pack_strings(genomes)
        return torch.from_numpy(arr).to(self.device), torch.from_numpy(lens).to(self.device)

    def _random_labels(self, k: int) -> tuple[torch.Tensor, torch.Tensor]:
        return world_ops.random_labels(self, k, _LABEL_LEN)

    def _find_free_random_positions(self, n_cells: int) -> torch.Tensor:
        return world_ops.free_positions(self, n_cells)

    def _get_molecule_map(self, n: int, size: int, init: str) -> torch.Tensor:
        shape = (n, size, size) if self._map_shape() == (size, size) else (n, *self._map_shape())
        if init == "zeros":
            return torch.zeros(*shape, dtype=self.map_dtype, device=self.device)
        if init == "randn":
            if self.map_dtype == torch.float32 and n * shape[1] * shape[2] <= (1 << 28):
                return (torch.randn(*shape, dtype=torch.float32, device=self.device) + 10.0).abs()
            # |N(10, 1)| drawn in chunks of rows: an HBM-sized map (hundreds of GB in fp16) has no
            # room for full-size fp32 temporaries
            mm = torch.empty(*shape, dtype=self.map_dtype, device=self.device)
            rows = max(1, (1 << 26) // shape[2])
            for i in range(n):
                for r in range(0, shape[1], rows):
                    blk = mm[i, r : r + rows]
                    blk.copy_((torch.randn(blk.shape, dtype=torch.float32, device=self.device) + 10.0).abs_())
            return mm
        raise ValueError(f"Didnt recognize mol_map_init={init}. Should be one of: 'zeros', 'randn'.")

    def _get_permeate(self, mol_perm_rate: float) -> float:
        return _permeation_factor(mol_perm_rate)

    def _get_diffuse(self, mol_diff_rate: float) -> tuple[float, float]:
        return _diffusion_weights(mol_diff_rate)

    def _i32_tensor(self, d: Any) -> torch.Tensor:
        return torch.tensor(d, device=self.device, dtype=torch.int32)

    def _f32_tensor(self, d: Any) -> torch.Tensor:
        return torch.tensor(d, device=self.device, dtype=torch.float32)

    # ------------------------------------------------------------------ observability
    def synchronize(self) -> None:
        """Settle everything issued so far: adopt a pending division count, issue and confirm the
        queued genome operations (replaying or rebuilding on the host where the device pipeline
        flagged it, redoing a speculative activity if that changed parameters), then wait for the
        device. After it the world's state is final and the GPU is idle (benchmarks stop their
        clock after this, so the last step's confirmation is inside the timed region)."""
        self._reconcile()
        if self._molmap.is_cuda:
            torch.cuda.synchronize(self._molmap.device)
            from magicsoup_amd.ops import hip_ops

            # (the device's error words -- grid barriers, look-back spins -- of everything issued
            # up to here, including an activity no division has confirmed yet)
            hip_ops.check_placement()

    def molecule_totals(self) -> torch.Tensor:
        """Per-species amounts, float64 ``(n_molecules, 2)`` on the world's device: column 0 the
        molecule map (a decomposed world: the whole global map, all-reduced -- collective), column 1
        all cells' intracellular molecules. Nothing waits on the device: on the GPU the map is read
        once by a native reduction with the pending diffusion correction / degradation applied on the
        fly (no full read + write pass to materialise it, as ``world.molecule_map`` would need), and
        one ``.tolist()`` gives all of it to the host. The reference's per-step molecule log
        (performance/run_simulation.py:102-113) is :meth:`molecule_means`."""
        self._reconcile()
        d = self.__dict__
        mm = d["_molmap"]
        m = self.n_molecules
        out = torch.zeros(m, 2, dtype=torch.float64, device=mm.device)
        R, C = int(mm.size(1)), int(mm.size(2))
        lo = 1 if getattr(self, "_exchange_map_halo", None) is not None else 0
        hi = R - lo
        if mm.is_cuda:
            from magicsoup_amd.ops import hip_ops

            tot = torch.zeros(m, dtype=torch.float64, device=mm.device)
            hip_ops._m().map_totals(m, R, C, lo, hi, mm.data_ptr(), hip_ops._p(d.get("_pending_corr")),
                                    hip_ops._p(d.get("_pending_scale")), hip_ops._mdt(mm), tot.data_ptr(),
                                    hip_ops._stream())
            out[:, 0] = tot
        else:
            out[:, 0] = self.molecule_map[:, lo:hi].double().sum(dim=(1, 2))
        if self.n_cells:
            out[:, 1] = self.cell_molecules.double().sum(dim=0)
        reduce = d.get("_allreduce_totals")
        if reduce is not None:
            reduce(out)
        return out

    def molecule_means(self) -> list[float]:
        """Per-species mean over all pixels and cells, (map total + cell total) / (pixels + cells) --
        what the reference's macro benchmark logs every step (performance/run_simulation.py:102-113,
        2m ``.item()`` synchronisations there; one here). Collective for a decomposed world."""
        t = self.molecule_totals()
        n = torch.tensor([float(self.n_cells)], dtype=torch.float64, device=t.device)
        reduce = self.__dict__.get("_allreduce_totals")
        if reduce is not None:
            reduce(n)
        v = torch.cat([t.sum(dim=1), n]).tolist()
        denom = float(self.map_size) ** 2 + v[-1]
        return [x / denom for x in v[:-1]]

    def enable_timings(self, sync: bool = False) -> None:
        """Time every public operation with HIP events (wall clock on CPU); read with
        :meth:`step_timings`. ``sync=True`` drains the device around each op (exact attribution of
        a kernel trace, at the cost of serialising host and device)."""
        from magicsoup_amd.utils.profiling import PhaseTimer

        self.__dict__["_timer"] = PhaseTimer(self.device, sync=sync)

    def disable_timings(self) -> None:
        self.__dict__.pop("_timer", None)

    def step_timings(self, reset: bool = True) -> dict[str, dict[str, float]]:
        """``{op: {"ms_total", "ms_mean", "n"}}`` since the last reset (resolves pending events)."""
        timer = self.__dict__.get("_timer")
        if timer is None:
            return {}
        out = timer.summary()
        if reset:
            self.enable_timings(sync=timer.sync)
        return out

    def set_debug_checks(self, on: bool = True) -> None:
        """Run :meth:`check_invariants` after every public operation (debug mode; syncs)."""
        self.__dict__["_debug_checks"] = bool(on)

    def check_invariants(self, where: str = "") -> None:
        """Raise ``RuntimeError`` if the population state is inconsistent: one cell per occupied
        pixel, ``cell_map`` matching ``cell_positions``, every per-cell column / string arena /
        kinetics row count equal to ``n_cells``."""
        n = self.n_cells
        R, C, r_lo, r_hi, _ = world_ops.geom(self)
        problems = []
        for name in self._cols:
            if getattr(self, name).size(0) != n:
                problems.append(f"{name} has {getattr(self, name).size(0)} rows")
        if len(self.cell_genomes) != n or len(self.cell_labels) != n:
            problems.append(f"{len(self.cell_genomes)} genomes / {len(self.cell_labels)} labels")
        if self.kinetics.__dict__.get("_ncells", 0) != n:
            problems.append(f"kinetics holds {self.kinetics.__dict__.get('_ncells', 0)} cells")
        pos = self.cell_positions.long()
        if n:
            inside = (pos[:, 0] >= r_lo) & (pos[:, 0] < r_hi) & (pos[:, 1] >= 0) & (pos[:, 1] < C)
            if not bool(inside.all()):
                problems.append(f"{int((~inside).sum())} positions outside the owned rows")
            else:
                if (pos[:, 0] * C + pos[:, 1]).unique().numel() != n:
                    problems.append("two cells share a pixel")
                if not bool(self.cell_map[pos[:, 0], pos[:, 1]].all()):
                    problems.append("cell_map is empty under a cell")
        occupied = int(self.cell_map[r_lo:r_hi].sum())
        if occupied != n:
            problems.append(f"cell_map has {occupied} occupied pixels for {n} cells")
        if problems:
            raise RuntimeError(f"World invariants violated{' after ' + where if where else ''}: " + "; ".join(problems))

    def health_flags(self) -> torch.Tensor:
        """Device int32 flags (no host sync): bit 0 = a non-finite value, bit 1 = a negative value,
        in the molecule map (bits 0/1) or in ``cell_molecules`` (bits 2/3)."""
        return world_ops.health_flags(self)

    def check_health(self) -> None:
        """Raise ``FloatingPointError`` if the molecule map or the cells hold NaN / Inf / negative
        amounts (one fused pass over the state, one sync)."""
        f = int(self.health_flags().item())
        if f:
            what = [txt for bit, txt in ((1, "non-finite map values"), (2, "negative map values"),
                                         (4, "non-finite cell molecules"), (8, "negative cell molecules")) if f & bit]
            raise FloatingPointError("unhealthy world state: " + ", ".join(what))

    def __repr__(self) -> str:
        return f"World(map_size:{self.map_size!r},abs_temp:{self.abs_temp!r},device:{self.device!r})"
