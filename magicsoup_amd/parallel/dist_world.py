"""A World domain-decomposed over the ranks of a torch.distributed group.

The reference simulates one map in one process (``python/magicsoup/world.py``); it has no multi-GPU
path. Here the map's x axis is cut into ``world_size`` strips of ``H = map_size / world_size`` rows,
one per rank (one process per MI355X, RCCL over xGMI; ``gloo`` for CPU runs). Each rank holds

* the molecule map of its strip plus one halo row on each side: ``(m, H + 2, map_size)``,
* the occupancy map in the same shape, and
* the cells whose pixels lie in its strip (local x in ``1..H``).

The global map is still a torus: rank 0's upper halo is rank ``N - 1``'s last row. Everything that
only touches a cell and its own pixel (integration, permeation, degradation, mutation, kill, spawn)
runs locally. What couples ranks:

* diffusion: the halo rows are refreshed before the stencil (two row exchanges per step) and the
  per-molecule mass totals of the correction are all-reduced so the global map conserves mass;
* integration: the equilibrium-damping early exit is the reference's ``torch.any`` over all cells
  (kinetics.py:837), so the four per-part iteration flags are MAX-all-reduced between parts;
* division into a neighbour's boundary row: before placement every rank sends each neighbour one
  byte per boundary column (occupied / dividing cell). The receiver copies the occupancy into its
  halo row and reserves its own free boundary pixels next to the neighbour's dividing cells, so
  the claims the two ranks make into the same row can never collide: children placed into a halo
  row are created on the owning rank from their records with no accept / reject round trip
  (``strip.py``, ``csrc/hip/dist.hip``). One host synchronisation reads the local winner counts and
  the neighbours' record headers together, as the single-GPU division reads its winner count.
* movement into a neighbour's boundary row: a claim protocol. Claims into a halo row are sent
  with the full cell record to the owner, which accepts a claim if the pixel is still free after its
  own placements and appends the cell; the claimer then drops the emigrant. A rejected cell does not
  move this step.
* recombination across a strip boundary: each rank receives its lower neighbour's boundary-row
  cells as ghosts, recombines pairs that include them, and sends the ghosts' new genomes back.

Communication goes through :mod:`magicsoup_amd.parallel.comm`: a native RCCL communicator driven
from C++ on the current HIP stream for GPU ranks (``nccl`` process groups), torch.distributed
(gloo) otherwise.

Per-cell RNG streams differ per rank, so a run is reproducible for a fixed rank count but not
bit-identical to a single-process run. Reserved boundary pixels make a child next to a strip
boundary avoid a pixel that a neighbour's dividing cell could claim in the same step; away from
strip boundaries placement is exactly the single-map algorithm.
"""
from __future__ import annotations

import copy
import os
import math
import random
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

from magicsoup_amd.models.world import World, _Deferred, _op
from magicsoup_amd.ops import world_ops
from magicsoup_amd.parallel import strip
from magicsoup_amd.parallel.comm import RcclComm, make_comm

_U8 = torch.uint8
# divide_cells over a mask as native calls when the exchanges go over RCCL (MS_NATIVE_DIVIDE=0: the
# Python protocol)
_NATIVE_DIVIDE = os.environ.get("MS_NATIVE_DIVIDE", "1") != "0"


def _pack(cols: list[torch.Tensor], k: int) -> torch.Tensor:
    """Byte-concatenate per-row columns into a (k, B) uint8 record block."""
    parts = [c.contiguous().view(_U8).reshape(k, -1) for c in cols]
    return torch.cat(parts, dim=1) if parts else torch.zeros(k, 0, dtype=_U8)


def _unpack(buf: torch.Tensor, specs: list[tuple[torch.dtype, int]]) -> list[torch.Tensor]:
    """Inverse of :func:`_pack` for columns of (dtype, elements per row)."""
    k = int(buf.size(0))
    out, o = [], 0
    for dt, n in specs:
        nb = n * torch.empty(0, dtype=dt).element_size()
        col = buf[:, o : o + nb].contiguous().view(dt)
        out.append(col.reshape(k) if n == 1 and dt != _U8 else col.reshape(k, n))
        o += nb
    return out


def _copy_maps(dst: World, src: World) -> None:
    """Give ``dst`` the genetics and kinetics parameter maps of ``src`` (on dst's device)."""
    dst.genetics = copy.deepcopy(src.genetics)
    kin, dev = dst.kinetics, torch.device(dst.device)
    for name in ("km_map", "vmax_map", "sign_map", "hill_map", "reaction_map", "transport_map", "effector_map"):
        mp = copy.deepcopy(getattr(src.kinetics, name))
        for attr, val in list(vars(mp).items()):
            if isinstance(val, torch.Tensor):
                setattr(mp, attr, val.to(dev))
        setattr(kin, name, mp)


# issue the boundary recombination's collective part at the recombinate_cells() call (MS_XB_EARLY=0:
# at the flush after the diffusion stencil, as before)
_XB_EARLY = os.environ.get("MS_XB_EARLY", "1") != "0"
# a lazy division's arrivals are built by the queued genome chain that follows (_divide_phase_b)
_ARRIVALS_MERGE = True
# the strip's kill / replicate step without a wait for the kill's survivor count (MS_STRIP_LAZY_KILL=0:
# the eager kill, then the lazy division)
_LAZY_KILL = os.environ.get("MS_STRIP_LAZY_KILL", "1") != "0"
# a lazy strip division's phase B after the diffusion stencil, on the side stream (MS_EARLY_STENCIL=0:
# phase B, then the stencil, on the compute stream), for strips of up to MS_EARLY_STENCIL_MAX_PX owned
# pixels: a 1448^2 strip (an 8-GPU rank's share of the flagship) gains ~12 %; on a 4096^2 strip the
# side stream's phase B + boundary recombination + chain outlast the stencil and the chain lands
# before the next activity instead of next to the stencil (no gain, profiles/r5/early_stencil/)
_EARLY_STENCIL = os.environ.get("MS_EARLY_STENCIL", "1") != "0"
_EARLY_STENCIL_MAX_PX = int(os.environ.get("MS_EARLY_STENCIL_MAX_PX", str(4 << 20)))
# ... and that stencil issued before the host waits for phase A's counts (0: after the wait)
_STENCIL_BEFORE_WAIT = os.environ.get("MS_STENCIL_BEFORE_WAIT", "1") != "0"


class DistributedWorld(World):
    """:class:`~magicsoup_amd.World` over the ranks of ``group`` (default: the whole job).

    Constructor arguments are those of ``World`` (``map_size`` is the global map size and must be a
    multiple of the number of ranks with at least 2 rows per rank). Every rank must call every
    method collectively (same order, same arguments apart from local cell indices).

    ``exact_global_exit`` (default True) keeps the reference's integrator semantics exactly: the
    equilibrium-damping early exit is decided over ALL cells of the job (kinetics.py:846), which costs
    one tiny MAX all-reduce per damping iteration (up to 12 per step). ``False`` lets every rank decide
    for its own cells (one fused integrator launch, no collectives; results then differ from a
    single-process world only where one rank would stop iterating while another continues).

    ``boundary_genome_cap`` (default 2048 nt): recombination across a strip boundary (both genomes
    of a pair straddling it) is computed on both ranks from exchanged genomes of at most this length;
    pairs with a longer genome recombine only within a strip.

    Local state (``cell_positions`` in local rows ``1..H``, ``molecule_map`` / ``cell_map`` with
    halo rows) is what the kernels work on; :meth:`global_positions`, :meth:`owned_molecule_map`,
    :meth:`gather` and :meth:`scatter_from` convert to and from the global picture.
    """

    def __init__(self, *args, group=None, exact_global_exit: bool = True, boundary_genome_cap: int = 2048,
                 strips: bool | None = None, **kwargs):
        if not dist.is_initialized():
            raise RuntimeError("DistributedWorld needs an initialised torch.distributed process group")
        g = self.__dict__
        g["group"] = group
        g["rank"] = dist.get_rank(group)
        g["world_size"] = dist.get_world_size(group)
        # strip protocol even on one rank ("virtual ranks": the rank is its own up / down neighbour,
        # halo rows are copies of its own boundary rows = the torus wrap); default: only for > 1 rank
        g["_strips"] = self.world_size > 1 if strips is None else bool(strips)
        map_size = kwargs.get("map_size", args[1] if len(args) > 1 else 128)
        n = self.world_size
        if map_size % n != 0 or map_size // n < 2:
            raise ValueError(f"map_size={map_size} must be a multiple of {n} ranks with >= 2 rows per rank")
        g["H"] = map_size // n
        g["row0"] = self.rank * self.H
        g["_up"] = dist.get_global_rank(group, (self.rank - 1) % n) if group is not None else (self.rank - 1) % n
        g["_down"] = dist.get_global_rank(group, (self.rank + 1) % n) if group is not None else (self.rank + 1) % n
        seed = kwargs.pop("seed", None)
        if seed is not None:
            kwargs["seed"] = int(seed) + 1_000_003 * self.rank  # independent streams per rank
        # Genetics (codon maps) and Kinetics (parameter maps) are random draws from Python's
        # `random`: every rank must hold the same ones, so build them from rank 0's stream
        # (with a seed, rank 0 derives it from its seed, so the maps and the strip-boundary
        # recombination streams of a seeded world do not depend on Python's global `random` state)
        if self.rank != 0:
            shared = [0]
        elif seed is not None:
            shared = [(int(seed) * 0x9E3779B97F4A7C15 + 0xD1B54A32D192ED03) & ((1 << 63) - 1)]
        else:
            shared = [random.getrandbits(63)]
        dist.broadcast_object_list(shared, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        own = random.getstate()
        random.seed(shared[0])
        try:
            super().__init__(*args, **kwargs)
        finally:
            random.setstate(own)
        g["_n_pix_global"] = map_size * map_size
        g["_stage"] = dist.get_backend(group) == "gloo" and torch.device(self.device).type == "cuda"
        g["_comm"] = make_comm(group, self.rank, n, self.device) if self._strips else None
        # a second communicator for the exchanges of genome ops issued on the side stream (deferred
        # recombination): RCCL operations of one communicator must not interleave across streams
        side = None
        if self._strips and isinstance(g["_comm"], RcclComm):
            side = make_comm(group, self.rank, n, self.device)
        g["_comm_side"] = side if side is not None else g["_comm"]
        # RCCL exchanges are stream-ordered device work: the halo exchange can run on a stream of its
        # own next to the interior stencil (ops/hip_ops.py diffuse); gloo exchanges are host-side
        g["_halo_async"] = isinstance(g["_comm"], RcclComm)
        g["migrated"] = {"divided_out": 0, "divided_in": 0, "moved_out": 0, "moved_in": 0, "rejected": 0}
        # strip-boundary recombination: a stream per boundary shared by its two ranks, genomes up to
        # `boundary_genome_cap` nt take part (longer ones recombine with cells of their own strip only)
        g["_xseed"] = int(shared[0]) ^ 0x5DEECE66D
        g["_xcall"] = 0
        g["boundary_genome_cap"] = max(16, (int(boundary_genome_cap) + 15) // 16 * 16)
        if self._strips:
            # hooks the op layer calls (World has them as None): halo refresh before the diffusion
            # stencil, MAX of the integrator's iteration flags, SUM of the diffusion mass totals
            g["_exchange_map_halo"] = self._do_exchange_map_halo
            if exact_global_exit:
                g["_allreduce_flags"] = self._do_allreduce_flags
            g["_allreduce_totals"] = self._do_allreduce_totals
            self._exchange_occupancy()  # first p2p call is collective on every rank
            self._do_exchange_map_halo()

    # ------------------------------------------------------------------ geometry
    def _map_shape(self) -> tuple[int, int]:
        if not self._strips:
            return self.map_size, self.map_size
        return self.H + 2, self.map_size

    def _geom(self) -> tuple[int, int, int, int, int]:
        S = self.map_size
        if not self._strips:
            return S, S, 0, S, 1
        return self.H + 2, S, 1, self.H + 1, 0

    @property
    def _lo(self) -> int:
        return 1 if self._strips else 0

    def global_positions(self) -> torch.Tensor:
        """Cell positions in global map coordinates (int32 (n, 2))."""
        pos = self.cell_positions.clone()
        pos[:, 0] += self.row0 - self._lo
        return pos

    def owned_molecule_map(self) -> torch.Tensor:
        """View (m, H, map_size) of the molecule map rows this rank owns."""
        mm = self.molecule_map
        return mm[:, self._lo : self._lo + self.H]

    def owned_cell_map(self) -> torch.Tensor:
        return self.cell_map[self._lo : self._lo + self.H]

    # ------------------------------------------------------------------ communication
    def _tensor_device(self) -> torch.device:
        return self._molmap.device

    def _exchange(self, to_up, to_down, from_down, from_up) -> None:
        """One neighbour exchange: ``to_up`` arrives at the upper neighbour as its ``from_down``,
        ``to_down`` at the lower one as its ``from_up``. ``None`` skips an op (the peer must skip
        the matching one)."""
        self._active_comm().exchange(to_up, to_down, from_down, from_up)

    def _active_comm(self):
        d = self.__dict__
        return d["_comm_side"] if d.get("_side_active") else d["_comm"]

    def _all_reduce(self, t: torch.Tensor, op) -> None:
        name = {dist.ReduceOp.SUM: "sum", dist.ReduceOp.MAX: "max", dist.ReduceOp.MIN: "min"}[op]
        self._active_comm().allreduce_(t, name)

    def _exchange_var(self, up: torch.Tensor | None, down: torch.Tensor | None, meta_up=(), meta_down=()):
        """Exchange variable-size uint8 record blocks (k, B) with both neighbours. ``meta_*`` are
        extra header ints (e.g. column widths). Returns ((block, meta) from down, (block, meta) from up)."""
        dev = self._tensor_device()
        nm = max(len(meta_up), len(meta_down))

        def hdr(block, meta):
            k, b = (0, 0) if block is None else (int(block.size(0)), int(block.size(1)))
            return torch.tensor([k, b, *meta, *([0] * (nm - len(meta)))], dtype=torch.int64, device=dev)

        h_up, h_dn = hdr(up, meta_up), hdr(down, meta_down)
        r_dn, r_up = torch.empty_like(h_up), torch.empty_like(h_up)
        self._exchange(h_up, h_dn, r_dn, r_up)
        hd, hu = r_dn.tolist(), r_up.tolist()
        s_up = up.reshape(-1) if up is not None and up.numel() else None
        s_dn = down.reshape(-1) if down is not None and down.numel() else None
        b_dn = torch.empty(hd[0] * hd[1], dtype=_U8, device=dev) if hd[0] * hd[1] else None
        b_up = torch.empty(hu[0] * hu[1], dtype=_U8, device=dev) if hu[0] * hu[1] else None
        self._exchange(s_up, s_dn, b_dn, b_up)

        def block(b, h):
            return torch.zeros(h[0], h[1], dtype=_U8, device=dev) if b is None else b.view(h[0], h[1])

        return (block(b_dn, hd), hd[2:]), (block(b_up, hu), hu[2:])

    def _halo_buffers(self) -> torch.Tensor:
        """(send up | send down | from down | from up) halo rows of every species, map dtype."""
        mm = self.__dict__["_molmap"]
        m, C = int(mm.size(0)), self.map_size
        sb = self.__dict__.get("_halo_bufs")
        if sb is None or sb.dtype != mm.dtype or sb.device != mm.device or sb.numel() != 4 * m * C:
            sb = torch.empty(4 * m * C, dtype=mm.dtype, device=mm.device)
            self.__dict__["_halo_bufs"] = sb
        return sb

    def _rccl_comm(self):
        """The native RCCL communicator of the main stream (None: exchanges go through torch)."""
        d = self.__dict__
        c = d.get("_comm")
        return c if isinstance(c, RcclComm) and not d.get("_side_active") else None

    def _do_exchange_map_halo(self) -> None:
        """Refresh the molecule-map halo rows from the neighbours' boundary rows (raw buffer: a
        pending degradation factor is identical on every rank and applied by the stencil). One pack
        launch, one grouped exchange, one unpack launch."""
        if not self._strips:
            return
        mm = self.__dict__["_molmap"]
        m, C = int(mm.size(0)), self.map_size
        sb = self._halo_buffers()
        s_up, s_dn, r_dn, r_up = (sb[i * m * C : (i + 1) * m * C] for i in range(4))
        strip.halo_pack(self, s_up, s_dn)
        self._exchange(s_up, s_dn, r_dn, r_up)
        strip.halo_unpack(self, r_up, r_dn)

    def _exchange_occupancy(self) -> None:
        if not self._strips:
            return
        cm = self.cell_map.view(_U8)
        H = self.H
        s_up, s_dn = cm[1].contiguous(), cm[H].contiguous()
        r_dn, r_up = torch.empty_like(s_up), torch.empty_like(s_up)
        self._exchange(s_up, s_dn, r_dn, r_up)
        cm[H + 1].copy_(r_dn)
        cm[0].copy_(r_up)

    def _rccl_handle(self) -> int | None:
        """Handle of the native RCCL communicator in use (None: exchanges go through torch /
        gloo), for native code that issues its collectives itself (hip_ops integrate_dist)."""
        c = self._active_comm()
        return c.handle if isinstance(c, RcclComm) and self.__dict__.get("_allreduce_flags") else None

    def _do_allreduce_flags(self, flags: torch.Tensor) -> None:
        self._all_reduce(flags, dist.ReduceOp.MAX)

    def _do_allreduce_totals(self, totals: torch.Tensor) -> None:
        self._all_reduce(totals, dist.ReduceOp.SUM)

    # ------------------------------------------------------------------ cell records
    def _records(self, cells: torch.Tensor, ys: torch.Tensor, child: bool) -> tuple[torch.Tensor, tuple[int, int]]:
        """Full records of ``cells`` landing on columns ``ys`` of a neighbour's boundary row: the
        child of a division (half the molecules, divisions + 1, lifetime 0) or the cell itself."""
        k = int(cells.numel())
        gw, lw = int(self._genomes.width), int(self._labels.width)
        if k == 0:
            return None, (gw, lw)
        mol = self.cell_molecules[cells]
        div = self.cell_divisions[cells]
        life = self.cell_lifetimes[cells]
        if child:
            mol = mol * 0.5
            div = div + 1
            life = torch.zeros_like(life)
        cols = [
            ys.to(torch.int32),
            self._genomes.lens[cells],
            self._labels.lens[cells],
            div.to(torch.int32),
            life.to(torch.int32),
            mol.to(torch.float32),
            self._labels.data[cells],
            self._genomes.rows_of(cells, gw),
        ]
        return _pack(cols, k), (gw, lw)

    def _unpack_records(self, buf: torch.Tensor, meta) -> dict:
        gw, lw = int(meta[0]), int(meta[1])
        m = self.n_molecules
        i32 = torch.int32
        ys, glen, llen, div, life, mol, lab, gen = _unpack(
            buf, [(i32, 1), (i32, 1), (i32, 1), (i32, 1), (i32, 1), (torch.float32, m), (_U8, lw), (_U8, gw)]
        )
        return dict(ys=ys, glen=glen, llen=llen, div=div, life=life, mol=mol, lab=lab, gen=gen)

    def _append_records(self, r: dict, row: int, keep: torch.Tensor) -> int:
        """Append the accepted records (bool mask ``keep``) as new cells on local row ``row``."""
        idx = torch.nonzero(keep).flatten()
        k = int(idx.numel())
        if k == 0:
            return 0
        n0 = self.n_cells
        self._grow(k)
        self._genomes.append_packed(r["gen"][idx], r["glen"][idx])
        self._labels.append_packed(r["lab"][idx], r["llen"][idx])
        new = torch.arange(n0, n0 + k, device=self.device)
        ys = r["ys"][idx]
        pos = torch.stack([torch.full_like(ys, row), ys], dim=1)
        self._place(new, pos)
        self.cell_molecules[new] = r["mol"][idx]
        self.cell_divisions[new] = r["div"][idx]
        self.cell_lifetimes[new] = r["life"][idx]
        self._update_params_rows(new)
        return k

    def _migrate(self, rec_up, rec_dn) -> tuple[torch.Tensor, torch.Tensor, int]:
        """Send claim records to the neighbours, accept / append incoming ones, and return the
        accept flags of our own claims (to up, to down) and the number of cells received."""
        (b_dn, m_dn), (b_up, m_up) = self._exchange_var(rec_up[0], rec_dn[0], rec_up[1], rec_dn[1])
        cmap = self.cell_map
        got = 0
        flags = {}
        arrived = {"up": 0, "dn": 0}
        # records from the upper neighbour land on our first row, from the lower one on our last
        for key, buf, meta, row in (("up", b_up, m_up, 1), ("dn", b_dn, m_dn, self.H)):
            if buf.size(0) == 0:
                flags[key] = None
                continue
            r = self._unpack_records(buf, meta)
            ys = r["ys"].long()
            ok = ~cmap[row, ys]
            got_k = self._append_records(r, row, ok)
            got += got_k
            arrived[key] = got_k
            flags[key] = ok.to(_U8)
        k_up = 0 if rec_up[0] is None else int(rec_up[0].size(0))
        k_dn = 0 if rec_dn[0] is None else int(rec_dn[0].size(0))
        dev = self._tensor_device()
        f_up = torch.empty(k_up, dtype=_U8, device=dev) if k_up else None
        f_dn = torch.empty(k_dn, dtype=_U8, device=dev) if k_dn else None
        # verdicts on records from up go back up (they arrive there as from-down), and vice versa
        self._exchange(flags["up"], flags["dn"], f_dn, f_up)
        acc_up = f_up.bool() if k_up else torch.zeros(0, dtype=torch.bool, device=dev)
        acc_dn = f_dn.bool() if k_dn else torch.zeros(0, dtype=torch.bool, device=dev)
        self.__dict__["_arrived"] = (arrived["up"], arrived["dn"])
        return acc_up, acc_dn, got

    # ------------------------------------------------------------------ physics overrides
    @_op("enzymatic_activity")
    def enzymatic_activity(self):
        """Integration (collective with ``exact_global_exit``). A rank whose strip holds no cells
        still takes part in the per-part MAX all-reduces of the iteration flags (with all-zero
        flags), so the ranks that do have cells see the same number of collectives."""
        hook = self.__dict__.get("_allreduce_flags")
        if self.n_cells == 0 and hook is not None:
            from magicsoup_amd.models.kinetics import _INCREMENTS, _TRIMS

            if self._molmap.is_cuda:
                from magicsoup_amd.ops import hip_ops

                hip_ops.integrate_idle(self, _TRIMS)
                return
            for _ in _TRIMS:
                hook(torch.zeros(len(_INCREMENTS), dtype=torch.int32, device=self._tensor_device()))
            return
        super().enzymatic_activity()

    # ------------------------------------------------------------------ lifecycle overrides
    @_op("divide_cells")
    def divide_cells_t(self, cell_idxs, lazy: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
        """Division (collective). Children landing in a neighbour's boundary row are created on
        that rank; the returned pairs cover local children only (counts in ``self.migrated``).
        ``lazy`` (GPU mask over RCCL, see :meth:`_divide_mask_native`): returns None and completes
        the division when the cell count is next needed; otherwise the pairs are returned.

        Protocol (module docstring): boundary marks -> reservations -> placement rounds ->
        winners split by destination row + record headers exchanged -> one synchronisation ->
        child records exchanged and appended; exporting parents keep half their molecules."""
        if not self._strips:
            return super().divide_cells_t(cell_idxs, lazy=lazy)
        from magicsoup_amd.ops.hip_ops import _scratch

        dev = self.device
        C, H, m = self.map_size, self.H, self.n_molecules
        gpu = self.cell_molecules.is_cuda
        # GPU mask over all cells: no index compaction (and no host round trip) before placement
        mask = None
        if (gpu and isinstance(cell_idxs, torch.Tensor) and cell_idxs.dtype == torch.bool
                and cell_idxs.numel() == self.n_cells and self.n_cells > 0):
            mask = cell_idxs.to(dev).contiguous().view(_U8)
            idxs, k = None, self.n_cells
        else:
            idxs = self._idx_tensor(cell_idxs)
            k = int(idxs.numel())
        if mask is not None and self._rccl_native():
            return self._divide_mask_native(mask, lazy=lazy)
        sc = _scratch(self)
        empty = torch.zeros(0, dtype=torch.long, device=dev)
        # 1. boundary bytes (occupied / dividing) to the neighbours; halo occupancy + reservations
        mk = sc.get("dv_marks", 4 * C, _U8, torch.device(dev))
        s_up, s_dn, r_dn, r_up = mk[:C], mk[C : 2 * C], mk[2 * C : 3 * C], mk[3 * C :]
        strip.marks(self, idxs, s_up, s_dn, mask=mask)
        self._exchange(s_up, s_dn, r_dn, r_up)
        strip.reserve(self, r_up, r_dn)
        # 2. placement (claims into the halo rows are final), winners by destination, headers
        lw, gw = int(self._labels.width), int(self._genomes.width)
        if gpu:
            from magicsoup_amd.ops import hip_ops

            cells = None if mask is not None else idxs.to(torch.int64).contiguous()
            kk = max(k, 1)
            dv = torch.device(dev)
            if mask is not None:
                result = hip_ops.place_rounds_raw(self, None, mask=mask)
            else:
                result = hip_ops.place_rounds_raw(self, cells) if k else sc.get("dv_res0", 1, torch.int64, dv)
            par = sc.get("dv_par", 3 * kk, torch.int64, dv)
            npos = sc.get("dv_npos", 6 * kk, torch.int32, dv).view(3 * kk, 2)
            st = sc.get("dv_status", 20, torch.int32, dv)
            strip.split_winners_gpu(self, cells, result, par, npos, st)
            self._exchange(st[4:8], st[8:12], st[16:20], st[12:16])
            hip_ops.guarded_sync()  # (peer failures raise instead of hanging the read-back)
            v = st.tolist()  # the one synchronisation: local winner counts + the neighbours' headers
            hip_ops.check_placement()
            n_loc, n_up, n_dn = v[0], v[1], v[2]
            hdr_up, hdr_dn = v[12:16], v[16:20]
            par_loc, pos_loc = par[:n_loc], npos[:n_loc]
            par_up, pos_up = par[kk : kk + n_up], npos[kk : kk + n_up]
            par_dn, pos_dn = par[2 * kk : 2 * kk + n_dn], npos[2 * kk : 2 * kk + n_dn]
        else:
            if k:
                parents, cpos = world_ops.divide_placement(self, idxs)
            else:
                parents, cpos = empty, torch.zeros(0, 2, dtype=torch.int32)
            i_loc, i_up, i_dn = strip.split_winners_cpu(self, parents, cpos)
            par_loc, pos_loc = parents[i_loc], cpos[i_loc]
            par_up, pos_up = parents[i_up], cpos[i_up]
            par_dn, pos_dn = parents[i_dn], cpos[i_dn]
            n_loc, n_up, n_dn = int(i_loc.numel()), int(i_up.numel()), int(i_dn.numel())
            # own children first: their pixels are taken before the neighbours' records land
            lp = pos_loc.long()
            self.cell_map[lp[:, 0], lp[:, 1]] = True
            hs = torch.tensor([n_up, lw, gw, m, n_dn, lw, gw, m], dtype=torch.int32)
            hr = torch.zeros(8, dtype=torch.int32)
            self._exchange(hs[:4], hs[4:], hr[4:], hr[:4])
            hdr_up, hdr_dn = hr[:4].tolist(), hr[4:].tolist()
        # 3. child records to the neighbours (exact sizes from the headers)
        B = strip.record_bytes(m, lw, gw)
        out = sc.get("dv_out", max(1, (n_up + n_dn) * B), _U8, torch.device(dev))
        out_up, out_dn = out[: n_up * B], out[n_up * B : (n_up + n_dn) * B]
        strip.pack(self, par_up, pos_up, par_dn, pos_dn, True, out_up, out_dn)
        b_up = hdr_up[0] * strip.record_bytes(m, hdr_up[1], hdr_up[2])
        b_dn = hdr_dn[0] * strip.record_bytes(m, hdr_dn[1], hdr_dn[2])
        inb = sc.get("dv_in", max(1, b_up + b_dn), _U8, torch.device(dev))
        in_up, in_dn = inb[:b_up], inb[b_up : b_up + b_dn]
        self._exchange(out_up, out_dn, in_dn, in_up)
        # 4. exporting parents keep half their molecules (every claim into a halo row is accepted),
        # 5. local children (rows n0 ..), then the arrivals
        n0 = self.n_cells
        if gpu:
            # par holds the three winner classes at [0, kk), [kk, 2kk), [2kk, 3kk)
            p_out = torch.cat([par_up, par_dn]) if n_up + n_dn else None
            children = self._commit_divisions_gpu(par_loc, pos_loc, n_loc, exporters=p_out)
        else:
            if n_up + n_dn:
                p_out = torch.cat([par_up, par_dn])
                world_ops.split_cells(self, p_out, p_out)
            children = torch.arange(n0, n0 + n_loc, device=dev)
            if n_loc:
                self._clone_rows(par_loc, children)
                self.cell_positions[n0 : n0 + n_loc] = pos_loc.to(torch.int32)
                world_ops.split_cells(self, par_loc, children)
        self._append_arrivals(hdr_up, in_up, hdr_dn, in_dn)
        # 6. halo rows empty, reservations released
        strip.clear(self)
        mig = self.migrated
        mig["divided_out"] += n_up + n_dn
        mig["divided_in"] += hdr_up[0] + hdr_dn[0]
        # what crossed a boundary, in record order (read by the global-index view, GlobalWorld)
        self.__dict__["_xfer"] = (par_up, par_dn, int(hdr_up[0]), int(hdr_dn[0]))
        return (par_loc if n_loc else empty), children

    def _rccl_native(self) -> bool:
        """Exchanges of the main stream go over the native RCCL communicator (the strip protocol
        can then run as native calls that issue their own exchanges)."""
        d = self.__dict__
        return not d.get("_side_active") and isinstance(d.get("_comm"), RcclComm) and _NATIVE_DIVIDE

    def _divide_mask_native(self, mask: torch.Tensor, lazy: bool = False) -> tuple[torch.Tensor, torch.Tensor] | None:
        """divide_cells_t over a GPU mask as two native calls around the one read-back of the
        counts (csrc/hip/fast.hip fast_dist_divide_a / _b): the same protocol, kernels and exchanges
        as the Python path below.

        ``lazy``: phase A (marks, reservations, placement, winners split by destination, headers
        exchanged) is issued and the call returns None; the read-back and phase B (child records
        exchanged, children committed, arrivals appended) follow when the cell count is next needed
        (:meth:`_resolve_count`: at the latest the next diffusion, before its stencil). What runs in
        between only queues genome operations or scales all capacity rows (degradation: halving a
        parent's molecules afterwards gives the same bits, the factor 0.5 is exact), so the result
        equals the eager protocol's, without the host waiting for the placement."""
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.hip_ops import _m, _p, _scratch, _stream

        comm = self.__dict__["_comm"]
        dev = self._tensor_device()
        n0, C = self.n_cells, self.map_size
        lw, gw = int(self._labels.width), int(self._genomes.width)
        fw = self._fast_world(n0)
        sc = _scratch(self)
        mk = sc.get("dv_marks", 4 * C, _U8, dev)
        par = sc.get("dv_par", 3 * n0, torch.int64, dev)
        npos = sc.get("dv_npos", 6 * n0, torch.int32, dev)
        st = sc.get("dv_status", 20, torch.int32, dev)
        host_st = self.__dict__.get("_dv_host_st")
        if host_st is None:
            host_st = self.__dict__["_dv_host_st"] = torch.zeros(20, dtype=torch.int32, pin_memory=True)
        seed, call = hip_ops._rng()
        _m().fast_dist_divide_a(fw, n0, _p(mask), comm.handle, comm.up, comm.down, seed, call, _p(mk), _p(par),
                                _p(npos), _p(st), lw, gw, host_st.data_ptr(), _stream())
        if lazy:
            from magicsoup_amd.ops.streams import NEvent

            self.__dict__["_count_pending"] = (n0, None, NEvent().record(), "strip", lw, gw)
            return None
        hip_ops.guarded_sync()  # (peer failures raise instead of hanging the read-back)
        return self._divide_phase_b(n0, lw, gw)

    def _kill_divide_native(self, n: int, mol: int, kill_below: float, divide_above: float, divide_cost: float,
                            kill_fraction: float) -> bool:
        """World.kill_divide_where on a strip whose exchanges go over RCCL, without waiting for the
        kill's survivor count (csrc/hip/fast.hip fast_dist_kill_divide_a): masks, payment, spill,
        the survivors' compaction and phase A of the division protocol over all ``n`` rows (rows past
        the survivors have a zero division mask) are one native call. The survivor count reaches the
        host with phase A's counts, at the one read-back of :meth:`_resolve_count`; ``last_kill`` is
        set there. Same draws, placement and rows as the eager kill followed by the lazy division
        (``MS_STRIP_LAZY_KILL=0``). Returns False when the eager path must run."""
        if not (_LAZY_KILL and self._strips and self._rccl_native()):
            return False
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.hip_ops import _m, _p, _scratch, _stream
        from magicsoup_amd.ops.streams import NEvent

        comm = self.__dict__["_comm"]
        dev = self._tensor_device()
        C = self.map_size
        lw, gw = int(self._labels.width), int(self._genomes.width)
        fw = self._fast_world(n)
        bufs = self.__dict__["_fw_bufs"]
        cap = int(bufs["sel"].numel())
        if bufs.get("kmask") is None or bufs["kmask"].numel() < cap:
            bufs["kmask"] = torch.empty(cap, dtype=torch.uint8, device=dev)
            bufs["dvmask"] = torch.empty_like(bufs["kmask"])
            bufs["dvmask2"] = torch.empty_like(bufs["kmask"])
        mm, corr = hip_ops.map_for_pixels(self)
        sc = _scratch(self)
        mk = sc.get("dv_marks", 4 * C, _U8, dev)
        par = sc.get("dv_par", 3 * n, torch.int64, dev)
        npos = sc.get("dv_npos", 6 * n, torch.int32, dev)
        st = sc.get("dv_status", 20, torch.int32, dev)
        host_st = self.__dict__.get("_dv_host_st")
        if host_st is None:
            host_st = self.__dict__["_dv_host_st"] = torch.zeros(20, dtype=torch.int32, pin_memory=True)
        # (the same draws in the same order as the eager path: the dilution's, then the placement's)
        mseed, mcall = hip_ops._rng() if kill_fraction > 0.0 else (0, 0)
        seed, call = hip_ops._rng()
        slot = _m().fast_dist_kill_divide_a(
            fw, n, mol, float(kill_below), float(divide_above), float(divide_cost), float(kill_fraction),
            mseed ^ 0x6A09E667F3BCC909, mcall, bufs["kmask"].data_ptr(), bufs["dvmask"].data_ptr(), mm.data_ptr(),
            hip_ops._mdt(mm), hip_ops._p(corr), comm.handle, comm.up, comm.down, seed, call, _p(mk), _p(par),
            _p(npos), _p(st), lw, gw, host_st.data_ptr(), _stream())
        self.__dict__["_count_pending"] = (n, None, NEvent().record(), "strip", lw, gw, int(slot))
        return True

    def _divide_phase_b(self, n0: int, lw: int, gw: int, defer_arrivals: bool = False, kk: int | None = None,
                        pairs: bool = True, stencil_first=None, _prepared: bool = False, stencil_before=None
                        ) -> tuple[torch.Tensor, torch.Tensor] | None:
        """Phase B of :meth:`_divide_mask_native` once phase A's counts are on the host (its pinned
        status copy is complete): records out, children in, arrivals appended and their parameter
        rows rebuilt on the device -- or, with ``defer_arrivals`` (a queued recombinate_cells() +
        mutate_cells() pair follows), built by that pair's device chain with the cells it changed
        (``_arrivals``, consumed by :meth:`_evolve`; one translation + build less per step)."""
        from magicsoup_amd.ops import genome_pipeline, hip_ops
        from magicsoup_amd.ops.hip_ops import _m, _p, _scratch, _stream

        comm = self.__dict__["_comm"]
        dev = self._tensor_device()
        m = self.n_molecules
        sc = _scratch(self)
        # (the stencil went out before the counts were read: the buffers as they were then)
        bufs0 = self._buffer_objs() if stencil_before is not None else None
        # kk: the row count phase A ran over (the cells before a lazy kill; par / npos offsets)
        kk = n0 if kk is None else int(kk)
        par = sc.get("dv_par", 3 * kk, torch.int64, dev)
        npos = sc.get("dv_npos", 6 * kk, torch.int32, dev)
        v = self.__dict__["_dv_host_st"].tolist()  # local winner counts + the neighbours' headers
        hip_ops.check_placement()
        n_loc, n_up, n_dn = v[0], v[1], v[2]
        hdr_up, hdr_dn = v[12:16], v[16:20]
        k_in = hdr_up[0] + hdr_dn[0]
        B = strip.record_bytes(m, lw, gw)
        out = sc.get("dv_out", max(1, (n_up + n_dn) * B), _U8, dev)
        b_in = hdr_up[0] * strip.record_bytes(m, hdr_up[1], hdr_up[2]) + hdr_dn[0] * strip.record_bytes(
            m, hdr_dn[1], hdr_dn[2])
        inb = sc.get("dv_in", max(1, b_in), _U8, dev)
        n_new = n0 + n_loc + k_in
        if k_in and not _prepared:
            for arena, wi in ((self._genomes, 2), (self._labels, 1)):
                w = max(int(hdr_up[wi]), int(hdr_dn[wi]), 1)
                if w > arena.width:
                    arena.reserve(n_new, w)
            # the arrivals' genomes go to fresh pool space (before the descriptor: a collection moves it)
            need = hdr_up[0] * ((int(hdr_up[2]) + 15) // 16 * 16) + hdr_dn[0] * ((int(hdr_dn[2]) + 15) // 16 * 16)
            self._genomes.ensure(need)
            self._genomes.top_ub += need
        fw = self._fast_world(n_new)
        zero_row = self.kinetics._zero_row()
        if stencil_first is not None:
            # the diffusion stencil first (it reads and writes only the molecule map, which phase B
            # does not touch: every capacity change above is done), then phase B on the side stream
            # over the side communicator, next to the stencil (see _diffuse_early)
            from magicsoup_amd.ops import world_ops
            from magicsoup_amd.ops.streams import NEvent, on_stream

            if stencil_before is None:
                before = NEvent().record()
                world_ops.diffuse(self)
            elif all(a is b for a, b in zip(self._buffer_objs(), bufs0)):
                before = stencil_before  # (the capacity steps above issued no device work)
            else:
                # a buffer was reallocated behind the stencil (rare): phase B waits for the copy
                before = NEvent().record()
            side = stencil_first
            before.wait(side.cuda_stream)
            self.__dict__["_side_active"] = True
            try:
                with on_stream(side):
                    return self._divide_phase_b(n0, lw, gw, defer_arrivals, kk, pairs, _prepared=True)
            finally:
                self.__dict__["_side_active"] = False
        comm = self._active_comm()
        _m().fast_dist_divide_b(fw, n0, comm.handle, comm.up, comm.down, _p(par), _p(npos), kk, n_loc, n_up, n_dn, lw,
                                gw, _p(out), _p(inb), hdr_up[0], hdr_up[1], hdr_up[2], hdr_dn[0], hdr_dn[1],
                                hdr_dn[2], _p(zero_row), _stream())
        self._adopt_count(n_new)
        if k_in:
            d = self.__dict__
            if (defer_arrivals and d.get("_arrivals") is None and k_in <= genome_pipeline.N_CAP
                    and genome_pipeline.enabled(self) and self.kinetics._P() > 0):
                d["_arrivals"] = (n0 + n_loc, k_in)
            else:
                self._rebuild_arrivals((n0 + n_loc, k_in))
        mig = self.migrated
        mig["divided_out"] += n_up + n_dn
        mig["divided_in"] += k_in
        self.__dict__["_xfer"] = (par[kk : kk + n_up], par[2 * kk : 2 * kk + n_dn], int(hdr_up[0]), int(hdr_dn[0]))
        if not pairs:  # (a lazy division's pairs are discarded: no arange launch for them)
            return None
        return par[:n_loc], torch.arange(n0, n0 + n_loc, device=self.device)

    def _buffer_objs(self) -> tuple:
        """The per-cell buffer objects a capacity step replaces when it reallocates (a new tensor
        object each time, see World._fast_world)."""
        g, lab, kd = self._genomes, self._labels, self.kinetics.__dict__
        return (g.data, g.off, g.lens, lab.data, lab.lens, kd.get("_slot_buf"), kd.get("_slot_spare"),
                self.__dict__.get("_cell_map"), *(c.buf for c in self._cols.values()))

    def _resolve_count(self, stencil_first=None, stencil_before=None) -> None:
        """Adopt a pending division: World's (a winner count) or a strip division issued with
        ``lazy=True`` (wait for its phase A only, then issue phase B, see _divide_mask_native). Queued
        genome operations then depend on phase B: their chains wait for it, not for the state when
        they were queued. ``stencil_first`` (a side stream, :meth:`_diffuse_early`): the diffusion
        stencil is issued before phase B, which goes to that stream."""
        d = self.__dict__
        pend = d.get("_count_pending")
        if pend is None or len(pend) < 4:
            return super()._resolve_count()
        from magicsoup_amd.ops import hip_ops

        n0, _, ev, _, lw, gw = pend[:6]
        hip_ops.guarded_sync(ev)
        # (the entry stays until the counts are read: a failure above leaves it for a retry)
        d["_count_pending"] = None
        kk = n0
        if len(pend) > 6:  # a lazy kill before phase A (_kill_divide_native): its survivors first
            n_k = int(hip_ops._m().status_read(pend[6])[0])
            d["last_kill"] = (n0, n_k)
            if n_k != n0:
                self._adopt_count(n_k)
            n0 = n_k
        # the genome ops queued since the division stay queued during phase B: its parameter
        # rebuild of the arrivals reconciles the world (Kinetics._sync), which would otherwise issue
        # them against the state before phase B
        queued = d.get("_deferred")
        d["_deferred"] = []
        pair = (_ARRIVALS_MERGE and queued is not None and len(queued) >= 2 and getattr(queued[0], "kind", None) == "rec"
                and getattr(queued[1], "kind", None) == "mut")
        try:
            self._divide_phase_b(n0, lw, gw, defer_arrivals=pair, kk=kk, pairs=False, stencil_first=stencil_first,
                                 stencil_before=stencil_before)
        finally:
            if queued:
                from magicsoup_amd.ops.streams import NEvent

                d["_deferred"] = queued + d["_deferred"]
                # (after phase B: on the side stream when it went there)
                d["_defer_event"] = NEvent().record(stencil_first.cuda_stream if stencil_first is not None else None)

    @_op("diffuse_molecules")
    def diffuse_molecules(self):
        """World's diffusion; a strip division issued lazily is completed first, so that its record
        exchange and commit are queued before the genome chains that follow it -- and, over RCCL with
        a side communicator of its own, after the stencil (:meth:`_diffuse_early`)."""
        if self._strips and self.__dict__.get("_count_pending") is not None:
            if self._early_stencil_ok():
                return self._diffuse_early()
            self._resolve_count()
            self._xb_pre_issue_queued()
        return super().diffuse_molecules()

    def _early_stencil_ok(self) -> bool:
        d = self.__dict__
        pend = d.get("_count_pending")
        return (_EARLY_STENCIL and pend is not None and len(pend) >= 6 and self._molmap.is_cuda
                and self.H * self.map_size <= _EARLY_STENCIL_MAX_PX
                and isinstance(d.get("_comm"), RcclComm) and isinstance(d.get("_comm_side"), RcclComm)
                and d["_comm_side"] is not d["_comm"] and not d.get("_side_active"))

    def _diffuse_early(self) -> None:
        """diffuse_molecules while a lazy strip division is pending, with the stencil before phase B.

        Phase B (record exchange, children and arrivals committed, halo rows cleared) touches the
        per-cell rows and the cell map, never the molecule map, and phase A's spill is queued before
        it; the stencil reads and writes only the map. So the stencil is issued first -- before the
        one wait for phase A's counts (``MS_STENCIL_BEFORE_WAIT``, default on: the host issues it
        while the counts travel) -- and phase B, the boundary recombination's collective part and the
        genome chains follow on the side stream over the side communicator, next to it: the device
        no longer idles while the host issues phase B and the chains (~150 us per flagship step as
        one virtual strip, profiles/r5/lazykill). Same kernels, draws and order per communicator on
        every rank, so the same results. The permeation waits for the side stream (it reads the
        committed children)."""
        from magicsoup_amd.ops import world_ops
        from magicsoup_amd.ops.hip_ops import _stream
        from magicsoup_amd.ops.streams import join

        d = self.__dict__
        side = d.get("_side_stream")
        if side is None:
            side = d["_side_stream"] = torch.cuda.Stream(device=self._genomes.data.device, priority=-1)
        main = _stream()
        from magicsoup_amd.ops.streams import NEvent

        if _STENCIL_BEFORE_WAIT:
            # the stencil before the wait for phase A's counts: it reads and writes only the map (phase
            # A's spill is queued before it), so the host issues it while the counts are on their way
            # instead of after them
            before = NEvent().record()
            world_ops.diffuse(self)
            self._resolve_count(stencil_first=side, stencil_before=before)
        else:
            self._resolve_count(stencil_first=side)
        from magicsoup_amd.ops.streams import on_stream

        with on_stream(side):
            self._xb_pre_issue_queued()
        if d.get("_deferred"):
            self._flush_deferred()
        join(main, side.cuda_stream)  # (phase B's rows before the permeation and what follows)
        if self.n_cells > 0:
            world_ops.permeate(self)

    def _xb_pre_issue_queued(self) -> None:
        """After a lazy division completed: issue the boundary recombination's collective part of
        the first queued recombinate_cells() now, before the stencil (what recombinate_cells() does
        at the call when no division is pending). Issued behind the stencil instead, its RCCL kernel
        waits for the stencil's workgroups (243 us at 4096^2) and the genome chain after it misses
        the stencil it should run next to (profiles/r4/s6/tfvirt_steps.txt)."""
        d = self.__dict__
        q = d.get("_deferred")
        if not (_XB_EARLY and q and getattr(q[0], "kind", None) == "rec" and q[0].args[1] is None
                and isinstance(d.get("_comm_side"), RcclComm)):
            return
        p = q[0].args[0]
        pre = self._xb_pre_issue(p)
        q[0] = _Deferred(lambda: self._recombinate_strips_all(p, pre), "rec", (p, pre))

    def _append_arrivals(self, hdr_up, in_up, hdr_dn, in_dn) -> None:
        """Append the records received from the upper (row 1) and lower (row H) neighbours as new
        cells and build their parameters (device genome pipeline on the GPU: no synchronisation)."""
        k = int(hdr_up[0]) + int(hdr_dn[0])
        if k == 0:
            return
        n1 = self.n_cells
        self._grow(k, zero=False)
        for arena, wi in ((self._genomes, 2), (self._labels, 1)):
            arena.reserve(n1 + k, max(int(hdr_up[wi]), int(hdr_dn[wi]), 1))
            arena.n = n1 + k
            arena.version += 1
        strip.unpack(self, n1, in_up, hdr_up, in_dn, hdr_dn)
        new = torch.arange(n1, n1 + k, device=self.device)
        from magicsoup_amd.ops import genome_pipeline

        if not (self.cell_molecules.is_cuda and genome_pipeline.rebuild_rows(self, new)):
            self._update_params_rows(new)

    def _split_by_row(self, rows: torch.Tensor):
        """Indices (in order) of entries whose local row is owned / the upper halo (0) / the lower
        halo (H + 1): one stable sort and one read-back."""
        if rows.numel() == 0:
            e = torch.zeros(0, dtype=torch.long, device=rows.device)
            return e, e, e
        cls = (rows == 0).to(torch.int8) + 2 * (rows == self.H + 1).to(torch.int8)
        order = torch.sort(cls, stable=True).indices
        c = torch.bincount(cls.to(torch.int64), minlength=3).tolist()
        return order[: c[0]], order[c[0] : c[0] + c[1]], order[c[0] + c[1] :]

    @_op("move_cells")
    def move_cells(self, cell_idxs=None):
        """Movement (collective). Cells moving into a neighbour's boundary row migrate to it."""
        if not self._strips:
            return super().move_cells(cell_idxs)
        if cell_idxs is None:
            cell_idxs = torch.arange(self.n_cells, device=self.device)
        idxs = self._idx_tensor(cell_idxs)
        dev = self.device
        self._exchange_occupancy()
        if idxs.numel():
            moved, npos = world_ops.move_placement(self, idxs)
            moved, npos = moved.to(dev), npos.to(dev)
        else:
            moved, npos = torch.zeros(0, dtype=torch.long, device=dev), torch.zeros(0, 2, dtype=torch.int32, device=dev)
        i_loc, i_up, i_dn = self._split_by_row(npos[:, 0])
        m_up, m_dn = moved[i_up], moved[i_dn]
        # local moves first, so the owner's arbitration sees its final occupancy (the placement
        # kernels already vacated their old pixels and marked the new ones)
        if i_loc.numel():
            mv = moved[i_loc]
            if npos.is_cuda:
                self.cell_positions[mv] = npos[i_loc]
            else:
                old = self.cell_positions[mv].long()
                self.cell_map[old[:, 0], old[:, 1]] = False
                self._place(mv, npos[i_loc])
        rec_up = self._records(m_up, npos[i_up, 1], False)
        rec_dn = self._records(m_dn, npos[i_dn, 1], False)
        acc_up, acc_dn, got = self._migrate(rec_up, rec_dn)
        self.cell_map[0] = False
        self.cell_map[self.H + 1] = False
        out_up, out_dn = m_up[acc_up], m_dn[acc_dn]
        gone = torch.cat([out_up, out_dn])
        self.__dict__["_xfer"] = (out_up, out_dn) + tuple(self.__dict__.pop("_arrived"))
        mig = self.migrated
        mig["moved_in"] += got
        mig["moved_out"] += int(gone.numel())
        mig["rejected"] += int(acc_up.numel() + acc_dn.numel() - gone.numel())
        if gone.numel():
            self._remove(gone)

    def _remove(self, idxs: torch.Tensor) -> None:
        """Drop cells that emigrated (free their pixels, no molecule spill)."""
        pos = self.cell_positions[idxs].long()
        self.cell_map[pos[:, 0], pos[:, 1]] = False
        keep = torch.ones(self.n_cells, dtype=torch.bool, device=self.device)
        keep[idxs] = False
        if keep.is_cuda:
            from magicsoup_amd.ops import hip_ops

            keep_idx, gone, _ = hip_ops.select(keep, "set", rest=True)
            self._compact(keep_idx, None, removed=gone)
        else:
            self._compact(torch.nonzero(keep).flatten(), keep)

    def reposition_cells(self, cell_idxs=None, uniform: bool = False):
        """Move cells to random free pixels. Default: pixels of this rank's strip (cells do not change
        rank; every rank may call it alone). ``uniform=True`` (collective, every rank calls it with
        its own local ``cell_idxs``): the reference semantics (world.py:575-608) -- the listed cells of
        all ranks leave their pixels and take uniformly random free pixels of the whole map, so a cell
        may move to another rank. One shared draw decides how many land on each rank (multivariate
        hypergeometric over the ranks' free pixels, the vacated ones included, as
        GlobalWorld.reposition_cells); which cells go where follows a shared permutation of the
        selected cells in rank order. Movers' records travel through one object all-gather (host);
        the stayers are repositioned inside the strip, the arrivals placed at random free pixels."""
        if not uniform or self.world_size == 1:
            return super().reposition_cells(cell_idxs)
        import numpy as np

        from magicsoup_amd.parallel.global_world import _CellRecord

        self._reconcile()
        n = self.n_cells
        if cell_idxs is None:
            idx = np.arange(n, dtype=np.int64)
        else:
            idx = np.unique(np.asarray(self._idx_tensor(cell_idxs).cpu(), dtype=np.int64))
        ws, me, g = self.world_size, self.rank, self.group
        info = [None] * ws
        dist.all_gather_object(info, (int(idx.size), int(self.H * self.map_size - n)), group=g)
        sel = [int(a) for a, _ in info]
        free = [int(b) + int(a) for a, b in info]  # (the selected cells' own pixels are vacated first)
        k = sum(sel)
        if k == 0:
            return
        calls = self.__dict__["_repos_calls"] = self.__dict__.get("_repos_calls", 0) + 1
        rng = np.random.default_rng([int(self._xseed) & ((1 << 63) - 1), calls, 0x5EED])  # (shared by the ranks)
        order = rng.permutation(k)
        counts = rng.multivariate_hypergeometric(np.asarray(free, dtype=np.int64), k)
        dest = np.empty(k, dtype=np.int64)
        lo = 0
        for r, c in enumerate(counts):
            dest[order[lo : lo + int(c)]] = r
            lo += int(c)
        first = int(sum(sel[:me]))
        mine = dest[first : first + idx.size]
        stay, leave = idx[mine == me], idx[mine != me]
        leave_g = np.arange(first, first + idx.size)[mine != me]  # (global order of the movers)
        records = []
        if leave.size:
            rows = torch.as_tensor(leave, device=self.device)
            genomes, labels = self.cell_genomes, self.cell_labels
            mol = self.cell_molecules[rows].detach().cpu()
            life = self.cell_lifetimes[rows].tolist()
            div = self.cell_divisions[rows].tolist()
            records = [(int(gi), int(dest[gi]), _CellRecord(genomes[int(r)], labels[int(r)], mol[i], life[i], div[i]))
                       for i, (gi, r) in enumerate(zip(leave_g.tolist(), leave.tolist()))]
            self._remove(torch.as_tensor(np.sort(leave), device=self.device))
        allrec = [None] * ws
        dist.all_gather_object(allrec, records, group=g)
        if stay.size:
            # (the rows of the stayers after the movers' removal: the rank of each among the kept)
            kept = np.setdiff1d(np.arange(n, dtype=np.int64), leave, assume_unique=True)
            super().reposition_cells(torch.as_tensor(np.searchsorted(kept, stay), device=self.device))
        arrivals = sorted((gi, rec) for rr in allrec for gi, d, rec in rr if d == me)
        if arrivals:
            placed = self.add_cells([rec.cell(self) for _, rec in arrivals])
            assert len(placed) == len(arrivals), "no free pixel left for an arriving cell"
        self.migrated["moved_out"] += int(leave.size)
        self.migrated["moved_in"] += len(arrivals)

    # ------------------------------------------------------------------ recombination
    @_op("recombinate_cells")
    def recombinate_cells(self, cell_idxs: list[int] | None = None, p: float = 1e-7):
        """Recombination between neighbouring cells (collective), including pairs that straddle a
        strip boundary. For all cells (the default): both ranks of a boundary exchange its rows'
        genome lengths, draw the boundary pairs' strand breaks from the boundary's shared stream,
        swap the involved genomes and compute the same recombinations; each keeps its own cell's
        result, committed after the pairs inside its strip (GPU: inside the device genome pipeline,
        no synchronisation). ``cell_idxs``: ghost-row protocol with host round trips."""
        if not self._strips:
            return super().recombinate_cells(cell_idxs, p)
        if cell_idxs is None and self._genomes.data.is_cuda and self._defer_genome_op():
            # queued like World's: every rank flushes at the same op, in call order, and its
            # exchanges then go through the side-stream communicator. The boundary part's collective
            # (lengths / event genomes exchanged) is issued now on the side stream (_xb_pre_issue)
            # (only as the first queued genome op: its genomes are then final for this call; a later
            # queued call computes its boundary part at the flush, after the earlier results)
            # (not while a lazy division is pending: its children and arrivals exist only after the
            # count is resolved, at the latest before the diffusion stencil; the chains follow it)
            early = (_XB_EARLY and not self.__dict__.get("_deferred") and self.__dict__.get("_count_pending") is None
                     and isinstance(self.__dict__.get("_comm_side"), RcclComm))
            pre = self._xb_pre_issue(p) if early else None
            self._defer(_Deferred(lambda: self._recombinate_strips_all(p, pre), "rec", (p, pre)))
            return
        self._reconcile()
        if cell_idxs is not None:
            return self._recombinate_subset(cell_idxs, p)
        self._recombinate_strips_all(p)

    def _evolve(self, rec, mut) -> int:
        """A queued recombinate_cells() + mutate_cells() pair: the boundary part's collective runs as
        for a recombination of its own (every rank, once per call), then the local pairs, the
        boundary results and the mutations go into one device chain (genome_pipeline.evolve with the
        boundary rows); if the pipeline declines, the recombination is issued on its own (1)."""
        if not self._strips:
            return super()._evolve(rec, mut)
        from magicsoup_amd.ops import genome_pipeline
        from magicsoup_amd.ops.genome_pipeline import K_CAP

        p, pre = rec.args
        if pre is None:
            self.__dict__["_xcall"] += 1
        x = pre if pre is not None else _BoundaryRecombination(self, p, K_CAP)
        arr = self.__dict__.pop("_arrivals", None)
        if self.n_cells >= 2 and genome_pipeline.evolve(self, p, *mut.args, extra=x, arrivals=arr):
            return 2
        if arr is not None:
            self._rebuild_arrivals(arr)
        self._recombinate_gpu(p, x)
        return 1

    def _rebuild_arrivals(self, arr: tuple[int, int]) -> None:
        """Parameter rows of the cells [first, first + count) (a division's arrivals)."""
        from magicsoup_amd.ops import genome_pipeline

        new = torch.arange(arr[0], arr[0] + arr[1], device=self.device)
        if not genome_pipeline.rebuild_rows(self, new):
            self._update_params_rows(new)

    def _flush_deferred(self) -> None:
        super()._flush_deferred()
        arr = self.__dict__.pop("_arrivals", None)
        if arr is not None:  # (the pair was not issued as one chain: e.g. fewer than 2 cells)
            self._rebuild_arrivals(arr)

    def _recombinate_strips_all(self, p: float, pre: "_BoundaryRecombination | None" = None) -> None:
        if pre is None:
            self.__dict__["_xcall"] += 1
        if self._genomes.data.is_cuda:
            self._recombinate_gpu(p, pre)
        else:
            self._recombinate_cpu(p)

    def _xb_pre_issue(self, p: float) -> "_BoundaryRecombination":
        """The collective part of the boundary recombination of a queued recombinate_cells(), issued
        at the call on the side stream (after the state so far, an event), instead of at the flush
        behind the diffusion stencil: there its RCCL kernel waited for the stencil's workgroups
        (~0.2 ms at 4096^2) and the genome chains after it no longer overlapped the stencil. Every
        rank issues it at the same call, so the side communicator's order is unchanged."""
        from magicsoup_amd.ops.genome_pipeline import K_CAP
        from magicsoup_amd.ops.streams import NEvent, on_stream

        d = self.__dict__
        side = d.get("_side_stream")
        if side is None:
            side = d["_side_stream"] = torch.cuda.Stream(device=self._genomes.data.device, priority=-1)
        NEvent().record().wait(side.cuda_stream)
        d["_side_active"] = True
        try:
            d["_xcall"] += 1
            with on_stream(side):
                return _BoundaryRecombination(self, p, K_CAP)
        finally:
            d["_side_active"] = False

    # ------------------------------------------------------------------ strip-boundary recombination
    def _xb_params(self, p: float):
        """(events kept per boundary E, slot width, seed of the boundary below, of the one above,
        call): identical on both ranks of every boundary."""
        C, W = self.map_size, self.boundary_genome_cap
        E = int(min(3 * C, 8 * math.ceil(3 * C * p * 2 * W) + 16))
        mix = 0x9E3779B97F4A7C15

        def bseed(upper_rank: int) -> int:
            return (self._xseed * mix + 0xD1B54A32D192ED03 * (upper_rank + 1)) & 0xFFFFFFFFFFFFFFFF

        return E, W, bseed(self.rank), bseed((self.rank - 1) % self.world_size), int(self._xcall)

    def _recombinate_gpu(self, p: float, pre: "_BoundaryRecombination | None" = None) -> None:
        from magicsoup_amd.ops import genome_pipeline, hip_ops
        from magicsoup_amd.ops.genome_pipeline import K_CAP

        x = pre if pre is not None else _BoundaryRecombination(self, p, K_CAP)
        if self.n_cells >= 2 and genome_pipeline.recombinate_all(self, p, extra=x):
            return
        # synchronous path (very high rates / fewer than 2 cells): local pairs, then the boundary
        if self.n_cells >= 2:
            changed = hip_ops.recombinate_all(self, p)
            if changed.numel():
                self._update_params_rows(changed)
        x.commit_standalone()

    def _recombinate_cpu(self, p: float) -> None:
        """Same protocol with numpy streams (CPU ranks: tests and rehearsals)."""
        from magicsoup_amd.ops.genome_pipeline import K_CAP

        E, W, seed_dn, seed_up, call = self._xb_params(p)
        C, H, n = self.map_size, self.H, self.n_cells
        g = self._genomes
        pos = self.cell_positions.long()
        own = {}
        for row in (1, H):
            o = torch.full((C,), -1, dtype=torch.long)
            sel = torch.nonzero(pos[:, 0] == row).flatten() if n else torch.zeros(0, dtype=torch.long)
            o[pos[sel, 1]] = sel
            own[row] = o
        lens_of = lambda o: torch.where(o >= 0, g.lens[o.clamp(min=0)].long(), torch.full_like(o, -1))  # noqa: E731
        mine_up = torch.cat([lens_of(own[1]), torch.tensor([g.width])]).to(torch.int32)
        mine_dn = torch.cat([lens_of(own[H]), torch.tensor([g.width])]).to(torch.int32)
        from_dn, from_up = torch.empty_like(mine_dn), torch.empty_like(mine_up)
        self._exchange(mine_up, mine_dn, from_dn, from_up)
        # events of the boundary below (we are its upper side, b = 0) and above (b = 1)
        events = []
        for b, la_row, lb_row, seed in ((0, mine_dn, from_dn, seed_dn), (1, from_up, mine_up, seed_up)):
            wx = min(W, int(mine_dn[C]), int(from_dn[C] if b == 0 else from_up[C]))
            ys = np.repeat(np.arange(C), 3)
            ds = np.tile(np.array([-1, 0, 1]), C)
            ok = (ds == 0) | ((ds == -1) & (C >= 2)) | ((ds == 1) & (C >= 3))
            yb = (ys + ds) % C
            la, lb = la_row[:C].numpy()[ys], lb_row[:C].numpy()[yb]
            valid = ok & (la >= 0) & (lb >= 0) & (la <= wx) & (lb <= wx) & (la + lb > 0)
            lam = np.where(valid, p * (la + lb), 0.0)
            k = np.random.default_rng([seed, call]).poisson(lam)
            k = np.minimum(np.minimum(k, K_CAP), np.maximum(la + lb, 0))
            items = np.nonzero(valid & (k > 0))[0][:E]
            for jb, i in enumerate(items):
                owner = int(own[H][ys[i]]) if b == 0 else int(own[1][yb[i]])
                events.append((b, jb, int(i), int(k[i]), owner))
        slot = 4 + W
        send = {b: torch.zeros(E * slot, dtype=_U8) for b in (0, 1)}
        for b, jb, i, k, c in events:
            L = int(g.lens[c])
            send[b][jb * slot : jb * slot + 4] = torch.tensor([L], dtype=torch.int32).view(_U8)
            send[b][jb * slot + 4 : jb * slot + 4 + L] = g.data[c, :L]
        recv_dn, recv_up = torch.empty_like(send[0]), torch.empty_like(send[1])
        self._exchange(send[1], send[0], recv_dn, recv_up)
        # pairs inside the strip first (committed), then the boundary results override
        changed = []
        if n >= 2:
            idxs = torch.arange(n)
            pairs = world_ops.neighbors(self, idxs, idxs)
            if pairs.size(0):
                changed.append(world_ops.recombinations(self, pairs, p).long())

        def genome(buf, jb):
            L = int(buf[jb * slot : jb * slot + 4].view(torch.int32))
            return buf[jb * slot + 4 : jb * slot + 4 + L].numpy().tobytes()

        results = {}
        for b, jb, i, k, c in events:
            upper, lower = (genome(send[0], jb), genome(recv_dn, jb)) if b == 0 else (genome(recv_up, jb),
                                                                                      genome(send[1], jb))
            r0, r1 = _recombine_pair(upper, lower, k, np.random.default_rng([seed_dn if b == 0 else seed_up, call, i]))
            results[c] = r0 if b == 0 else r1  # last event per cell wins
        if results:
            rows = sorted(results)
            from magicsoup_amd.models.strings import pack_strings

            arr, lens = pack_strings([results[r].decode("ascii") for r in rows])
            g.set_rows(torch.tensor(rows, dtype=torch.long), torch.from_numpy(arr), torch.from_numpy(lens))
            changed.append(torch.tensor(rows, dtype=torch.long))
        if changed:
            self._update_params_rows(torch.unique(torch.cat(changed)))

    def _recombinate_subset(self, cell_idxs, p: float) -> None:
        """``recombinate_cells(cell_idxs)`` (collective): a rank recombines its last-row cells with
        ghosts of the lower neighbour's first row and returns the ghosts' new genomes to their owner."""
        dev = self.device
        n = self.n_cells
        pos = self.cell_positions
        # ghosts for the upper neighbour: our first-row cells
        first = torch.nonzero(pos[:, 0] == 1).flatten() if n else torch.zeros(0, dtype=torch.long, device=dev)
        if cell_idxs is not None:
            allowed = torch.zeros(n, dtype=torch.bool, device=dev)
            allowed[self._idx_tensor(cell_idxs)] = True
            first = first[allowed[first]]
        k = int(first.numel())
        send = None
        if k:
            send = _pack([first.to(torch.int32), pos[first, 1], self._genomes.lens[first],
                          self._genomes.rows_of(first, int(self._genomes.width))], k)
        (g_buf, g_meta), _ = self._exchange_var(send, None, (int(self._genomes.width),), (0,))
        ng = int(g_buf.size(0))
        changed_local = torch.zeros(0, dtype=torch.long, device=dev)
        upd = None
        if n + ng >= 2:
            idxs = torch.arange(n, device=dev) if cell_idxs is None else self._idx_tensor(cell_idxs)
            if ng:
                gi, gy, gl, gd = _unpack(g_buf, [(torch.int32, 1), (torch.int32, 1), (torch.int32, 1), (_U8, int(g_meta[0]))])
                gpos = torch.stack([torch.full_like(gy, self.H + 1), gy], dim=1)
                all_pos = torch.cat([pos, gpos]).contiguous()
                to = torch.cat([idxs, torch.arange(n, n + ng, device=dev)])
                pairs = world_ops.neighbors(self, idxs, to, pos=all_pos) if idxs.numel() else None
                self._genomes.append_packed(gd, gl)  # ghost rows n .. n+ng-1 (temporary)
            else:
                pairs = self.get_neighbors_t(idxs) if idxs.numel() else None
            try:
                if pairs is not None and pairs.size(0):
                    changed = world_ops.recombinations(self, pairs.to(dev), p).to(dev)
                    changed_local = changed[changed < n]
                    cg = changed[changed >= n] - n
                    if cg.numel():
                        rows = cg + n
                        upd = _pack([gi[cg], self._genomes.lens[rows], self._genomes.rows_of(rows, int(self._genomes.width))],
                                    int(cg.numel()))
            finally:
                if ng:
                    self._genomes.n = n
                    self._genomes.version += 1
        # ghost updates go back down to their owners
        _, (u_buf, u_meta) = self._exchange_var(None, upd, (0,), (int(self._genomes.width),))
        if u_buf.size(0):
            ui, ul, ud = _unpack(u_buf, [(torch.int32, 1), (torch.int32, 1), (_U8, int(u_meta[0]))])
            rows = ui.long()
            self._genomes.set_rows(rows, ud, ul)
            changed_local = torch.cat([changed_local, rows])
        if changed_local.numel():
            self._update_params_rows(torch.unique(changed_local))

    # ------------------------------------------------------------------ global views / persistence
    def gather(self, dst: int = 0) -> World | None:
        """Assemble the global state as a single-process CPU :class:`World` on rank ``dst``
        (``None`` elsewhere). Proteomes are re-derived from the genomes."""
        mm = self.owned_molecule_map().cpu()
        part = {
            "genomes": self.cell_genomes.tolist(),
            "labels": self.cell_labels.tolist(),
            "pos": self.global_positions().cpu(),
            "mol": self.cell_molecules.cpu(),
            "life": self.cell_lifetimes.cpu(),
            "div": self.cell_divisions.cpu(),
            "mm": mm,
        }
        parts = [None] * self.world_size if self.rank == dst else None
        dist.gather_object(part, parts, dst=dist.get_global_rank(self.group, dst) if self.group else dst, group=self.group)
        if self.rank != dst:
            return None
        w = World(
            chemistry=self.chemistry,
            map_size=self.map_size,
            abs_temp=self.abs_temp,
            mol_map_init="zeros",
            start_codons=self.genetics.start_codons,
            stop_codons=self.genetics.stop_codons,
            device="cpu",
        )
        _copy_maps(w, self)
        w.molecule_map = torch.cat([q["mm"] for q in parts], dim=1)
        genomes = [g for q in parts for g in q["genomes"]]
        n = len(genomes)
        if n:
            w._grow(n)
            w._genomes.append_strings(genomes)
            w._labels.append_strings([lab for q in parts for lab in q["labels"]])
            pos = torch.cat([q["pos"] for q in parts])
            w._place(torch.arange(n), pos)
            w.cell_molecules[:] = torch.cat([q["mol"] for q in parts])
            w.cell_lifetimes[:] = torch.cat([q["life"] for q in parts])
            w.cell_divisions[:] = torch.cat([q["div"] for q in parts])
            w._update_params_rows(torch.arange(n))
        return w

    def adopt_maps(self, world: World) -> None:
        """Use the genetics (codon maps) and kinetics parameter maps of ``world``."""
        _copy_maps(self, world)

    def scatter_from(self, world: World, maps: bool = True, params: bool = True) -> None:
        """Replace this rank's state by its strip of a global ``world`` (same on every rank);
        with ``maps`` also adopt its genetics / kinetics maps."""
        S, H, lo = self.map_size, self.H, self._lo
        if world.map_size != S:
            raise ValueError("map sizes differ")
        if maps:
            self.adopt_maps(world)
        gpos = world.cell_positions.long().cpu()
        mine = torch.nonzero((gpos[:, 0] >= self.row0) & (gpos[:, 0] < self.row0 + H)).flatten()
        k = int(mine.numel())
        genomes = labels = None
        if k:
            from magicsoup_amd.models.strings import pack_strings

            sel = mine.tolist()
            arr, lens = pack_strings(world._genomes.to_strings(sel))
            genomes = (torch.from_numpy(arr), torch.from_numpy(lens))
            arr, lens = pack_strings(world._labels.to_strings(sel))
            labels = (torch.from_numpy(arr), torch.from_numpy(lens))
        lpos = gpos[mine].clone()
        lpos[:, 0] += lo - self.row0
        cols = {name: getattr(world, name)[mine.to(getattr(world, name).device)]
                for name in ("cell_molecules", "cell_lifetimes", "cell_divisions")}
        self._adopt_strip(world.molecule_map[:, self.row0 : self.row0 + H], genomes, labels, lpos.to(torch.int32), cols,
                          params=params)

    def _adopt_strip(self, owned_map: torch.Tensor, genomes, labels, lpos: torch.Tensor, cols: dict,
                     params: bool = True) -> None:
        """Replace this rank's state: ``owned_map`` (m, H, map_size) becomes the owned rows of the
        molecule map; the cells -- packed genome / label rows + lengths, local positions, and the
        ``cell_molecules`` / ``cell_lifetimes`` / ``cell_divisions`` rows -- replace the local ones
        (parameters rebuilt on the device unless ``params`` is False); halos are refreshed
        (collective in strips)."""
        H, lo = self.H, self._lo
        self.kill_cells_local_all()
        mm = self.__dict__["_molmap"]
        mm.zero_()
        mm[:, lo : lo + H] = owned_map.to(mm.device, mm.dtype)
        self.__dict__["_pending_scale"] = None
        self.__dict__["_pending_corr"] = None
        k = int(lpos.size(0))
        if k:
            self._grow(k)
            self._genomes.append_packed(*genomes)
            self._labels.append_packed(*labels)
            new = torch.arange(k, device=self.device)
            self._place(new, lpos.to(torch.int32))
            for name, t in cols.items():
                getattr(self, name)[:] = t.to(self.device)
            if params:
                self._update_params_rows(new)
        if self._strips:
            self._do_exchange_map_halo()

    # ------------------------------------------------------------------ global index space
    def _gather_ints(self, v: int) -> list[int]:
        t = torch.zeros(self.world_size, dtype=torch.int64)
        t[self.rank] = int(v)
        t = t.to(self._tensor_device()) if not self._stage else t
        self._all_reduce(t, dist.ReduceOp.SUM)
        return [int(x) for x in t.cpu().tolist()]

    def n_cells_global(self) -> int:
        """Collective: number of cells over all ranks."""
        return sum(self._gather_ints(self.n_cells))

    def global_index_offset(self) -> int:
        """Collective: global index of this rank's local cell 0 (cells are numbered rank by rank)."""
        return sum(self._gather_ints(self.n_cells)[: self.rank])

    def spawn_cells_global(self, genomes: list[str]) -> list[int]:
        """Collective; every rank passes the same ``genomes``. Places them uniformly over the free
        pixels of the WHOLE map (reference world.py:287-341 semantics on the global torus): the
        number landing on each rank is a multivariate-hypergeometric draw over the ranks' free pixel
        counts (shared seed, identical on every rank), each rank then spawns its share uniformly in
        its strip. More genomes than free pixels: a random subset is kept. Returns the local
        indices of the cells this rank received."""
        free = self._gather_ints(self.H * self.map_size - self.n_cells)
        seed = [random.getrandbits(63) if self.rank == 0 else 0]
        dist.broadcast_object_list(seed, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0,
                                   group=self.group)
        rng = np.random.default_rng(seed[0])
        n = min(len(genomes), sum(free))
        order = rng.permutation(len(genomes))[:n]
        counts = rng.multivariate_hypergeometric(np.asarray(free, dtype=np.int64), n) if n else [0] * len(free)
        lo = int(np.sum(counts[: self.rank]))
        mine = [genomes[int(i)] for i in order[lo : lo + int(counts[self.rank])]]
        return self.spawn_cells(mine) if mine else []

    def global_view(self):
        """Collective: a :class:`~magicsoup_amd.parallel.GlobalWorld` over this world (the
        reference ``World`` API with global cell indices)."""
        from magicsoup_amd.parallel.global_world import GlobalWorld

        return GlobalWorld(self)

    def kill_cells_local_all(self) -> None:
        """Remove every local cell without spilling molecules (state reset)."""
        if self.n_cells:
            self._remove(torch.arange(self.n_cells, device=self.device))

    def save_state(self, statedir: Path, assemble: bool = True):
        """Collective. Every rank writes its shard under ``statedir/shards/`` at the same time, from
        its own device memory (utils.checkpoint.save_shard: owned map rows, its cells with global
        positions, genomes / labels as packed bytes, its random streams); with ``assemble`` rank 0
        then writes the reference layout from the shards (``cells.fasta``, ``*.pt``, as a
        single-process world's ``save_state``). ``assemble=False`` skips that step for worlds
        whose global map one host should not hold (``checkpoint.assemble_state`` does it offline)."""
        from magicsoup_amd.utils import checkpoint

        statedir = Path(statedir)
        if self.rank == 0:
            # (a stale shard set of another rank count would make the directory ambiguous)
            import shutil

            root = statedir / checkpoint.SHARD_DIR
            if root.is_dir():
                for p in root.iterdir():
                    if not p.name.endswith(f"_of{self.world_size:04d}"):
                        shutil.rmtree(p)
        dist.barrier(group=self.group)
        checkpoint.save_shard(self, statedir)
        dist.barrier(group=self.group)
        if assemble and self.rank == 0:
            checkpoint.assemble_state(statedir)
        dist.barrier(group=self.group)

    def save_state_gathered(self, statedir: Path):
        """Collective: rank 0 assembles the global world on the CPU (:meth:`gather`: every genome
        re-translated there) and writes it; kept as the oracle of the sharded :meth:`save_state`."""
        w = self.gather()
        if w is not None:
            w.save_state(Path(statedir))
        dist.barrier(group=self.group)

    def load_state(self, statedir: Path, ignore_cell_params: bool = False, restore_rng: bool = False) -> str:
        """Collective. Each rank loads its own shard when the state has shards of this rank count
        (``restore_rng`` then restores the rank's random streams: a run resumes exactly), otherwise
        its strip of the reference files -- map rows memory-mapped, its cells picked from the FASTA
        -- with no CPU world. Returns the source used (``"shard"`` / ``"reference"``)."""
        from magicsoup_amd.utils import checkpoint

        self._reconcile()
        return checkpoint.load_strip(self, Path(statedir), ignore_cell_params=ignore_cell_params,
                                     restore_rng=restore_rng)

    def close(self) -> None:
        """Release the communicator (collective). The world cannot exchange afterwards."""
        d = self.__dict__
        side = d.get("_comm_side")
        if side is not None and side is not d.get("_comm"):
            side.close()
        c = d.get("_comm")
        if c is not None:
            c.close()

    def __getstate__(self):
        raise TypeError("a DistributedWorld is bound to its process group; use gather() or save_state()")

    def __repr__(self) -> str:
        return (
            f"DistributedWorld(map_size:{self.map_size!r},rank:{self.rank}/{self.world_size},"
            f"rows:{self.row0}..{self.row0 + self.H - 1},device:{self.device!r})"
        )


def _recombine_pair(a: bytes, b: bytes, k: int, rng) -> tuple[bytes, bytes]:
    """Recombination of two genomes with k strand breaks (reference rust/mutations.rs:78-154): cut
    both strands at k sorted positions, shuffle the k + 2 parts, split at a random index."""
    n0, nb = len(a), len(a) + len(b)
    cuts = sorted(int(c) for c in rng.choice(nb, size=min(k, nb), replace=False)) if nb else []
    parts, start, src = [], 0, a
    for c in cuts:
        if c < n0:
            parts.append(a[start:c])
            start = c
    parts.append(a[start:])
    start = 0
    for c in cuts:
        if c >= n0:
            parts.append(b[start : c - n0])
            start = c - n0
    parts.append(b[start:])
    order = rng.permutation(len(parts))
    parts = [parts[o] for o in order]
    split = int(rng.integers(0, len(parts)))
    return b"".join(parts[:split]), b"".join(parts[split:])


class _BoundaryRecombination:
    """GPU side of the strip-boundary recombination (dist.hip xb_*). The constructor is the
    collective part (lengths and event genomes exchanged, no synchronisation); :meth:`apply` writes
    this rank's results after the strip's own pair results inside the genome pipeline."""

    def __init__(self, world: DistributedWorld, p: float, kcap: int):
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.hip_ops import _m, _p, _scratch, _stream

        self.world = w = world
        E, W, self.seed_dn, self.seed_up, self.call = world._xb_params(p)
        self.E, self.W = E, W
        self.rows = 2 * E
        C, H, n = w.map_size, w.H, w.n_cells
        dev = w._genomes.data.device
        sc = _scratch(w)
        st = _stream()
        g = w._genomes
        R = H + 2
        idx_map = hip_ops._index_map(w, R * C, dev)
        hip_ops._ensure_world_layout(w)
        lens = sc.get("xb_lens", 4 * (C + 1), torch.int32, dev)
        own = sc.get("xb_own", 2 * C, torch.int32, dev)
        nev = 5 * 2 * E + 4
        ev = sc.bufs.get("xb_ev")
        if ev is None or ev.numel() != nev or ev.device != dev:
            ev = sc.bufs["xb_ev"] = torch.zeros(nev, dtype=torch.int32, device=dev)  # counts[3]: dropped total
        self.ev = ev
        slot = 4 + W
        sl = sc.get("xb_slots", 4 * E * slot, torch.uint8, dev)
        self.slots_dn, self.slots_up, self.recv_dn, self.recv_up = (sl[i * E * slot : (i + 1) * E * slot] for i in range(4))
        comm = w._active_comm()
        if isinstance(comm, RcclComm):
            # index map, lengths exchange, events, event-genome exchange: one native call (dist.hip)
            _m().xb_begin(C, H, n, _p(w.cell_positions), _p(idx_map), _p(g.lens), _p(g.data), _p(g.off), int(g.width),
                          _p(lens),
                          _p(own), E, W, float(p), int(kcap), self.seed_dn, self.seed_up, self.call, _p(ev), _p(sl),
                          comm.handle, comm.up, comm.down, st)
        else:
            _m().index_map(n, _p(w.cell_positions), C, _p(idx_map), False, st)
            mine_up, mine_dn, from_dn, from_up = (lens[i * (C + 1) : (i + 1) * (C + 1)] for i in range(4))
            _m().xb_prep(C, H, n, _p(w.cell_positions), _p(idx_map), _p(g.lens), int(g.width), _p(mine_up),
                         _p(mine_dn), _p(own[:C]), _p(own[C:]), st)
            w._exchange(mine_up, mine_dn, from_dn, from_up)
            _m().xb_events(C, E, W, float(p), int(kcap), self.seed_dn, self.seed_up, self.call, _p(mine_dn),
                           _p(from_dn), _p(mine_up), _p(from_up), _p(own[:C]), _p(own[C:]), _p(g.data), _p(g.off),
                           _p(ev), _p(self.slots_dn), _p(self.slots_up), st)
            w._exchange(self.slots_up, self.slots_dn, self.recv_dn, self.recv_up)
        self.parts = sc.get("xb_parts", 2 * E * (kcap + 2) * 3, torch.int32, dev)
        self.kcap = kcap

    def apply(self, pair_count, out, out_w, out_len, out_rows, nres) -> None:
        """Write this rank's boundary results after the ``2 * *pair_count`` local result rows
        (device pointers or tensors; ``pair_count`` None: from row 0) and the row total to ``nres``."""
        from magicsoup_amd.ops.hip_ops import _m, _scratch, _stream

        def ptr(x):
            return 0 if x is None else (x if isinstance(x, int) else x.data_ptr())

        other = _scratch(self.world).get("xb_other", 2 * self.E * int(out_w), torch.uint8, self.ev.device)
        _m().xb_apply(self.world.map_size, self.E, self.W, self.seed_dn, self.seed_up, self.call, ptr(self.ev),
                      ptr(self.slots_dn), ptr(self.slots_up), ptr(self.recv_dn), ptr(self.recv_up), ptr(self.parts),
                      self.kcap + 2, ptr(pair_count), ptr(out), int(out_w), ptr(out_len), ptr(out_rows), ptr(other),
                      ptr(nres), _stream())

    def commit_standalone(self) -> None:
        """Synchronous commit of this rank's boundary results (when the pipeline did not run)."""
        from magicsoup_amd.ops import hip_ops
        from magicsoup_amd.ops.hip_ops import _scratch

        w = self.world
        dev = w._genomes.data.device
        sc = _scratch(w)
        out_w = 2 * self.W
        out = sc.get("xb_out", 2 * self.E * out_w, torch.uint8, dev)
        out_len = sc.get("xb_out_len", 2 * self.E, torch.int32, dev)
        out_rows = sc.get("xb_out_rows", 2 * self.E, torch.int64, dev)
        nres = sc.get("xb_nres", 1, torch.int32, dev)
        self.apply(None, out, out_w, out_len, out_rows, nres)
        k = int(nres.item())
        if k == 0:
            return
        rows = out_rows[:k]
        need = int(out_len[:k].max().item())
        changed = hip_ops._arena_commit(w._genomes, rows, out.view(-1, out_w)[:k], out_len[:k], need, dedupe=True,
                                        owner=w)
        w._update_params_rows(torch.unique(changed))

    def dropped(self) -> int:
        return int(self.ev[-1].item())
