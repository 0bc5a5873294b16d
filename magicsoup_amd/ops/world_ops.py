"""Device dispatch of the World's bulk operations.

Every function takes the world and works on its device-resident state. HIP tensors go to the
gfx950 kernels in :mod:`magicsoup_amd.ops.hip_ops` (no fallback); CPU tensors go to the OpenMP host
core plus a few plain tensor ops for trivially elementwise work.
"""
from __future__ import annotations

import string

import numpy as np
import torch

from magicsoup_amd.ops import native

_LABEL_ALPHABET = torch.tensor(
    list((string.ascii_uppercase + string.ascii_lowercase + string.digits).encode("ascii")), dtype=torch.uint8
)
_gen_cpu = torch.Generator(device="cpu")
_gen_cpu.manual_seed(torch.initial_seed() & 0xFFFFFFFF)


def _is_gpu(world) -> bool:
    # the raw buffer: reading `molecule_map` would apply a pending (fused) degradation
    return world.__dict__["_molmap"].is_cuda


def _hip():
    from magicsoup_amd.ops import hip_ops

    return hip_ops


def set_seed(seed: int, device=None) -> None:
    """Seed the placement / mutation / label streams of both native cores."""
    native.host().set_seed(int(seed))
    _gen_cpu.manual_seed(int(seed) & 0xFFFFFFFFFFFF)
    if device is not None and torch.device(device).type == "cuda":
        _hip().set_seed(int(seed))


def _np(t: torch.Tensor):
    return t.detach().cpu().numpy()


def geom(world) -> tuple[int, int, int, int, int]:
    """(rows, cols, first owned row, end of owned rows, x wraps) of a world's local map. A whole
    map wraps in x; a strip of a domain-decomposed world (magicsoup_amd.parallel) has one halo row
    on each side and does not."""
    g = getattr(world, "_geom", None)
    if g is not None:
        return g()
    S = int(world.map_size)
    return S, S, 0, S, 1


def _halo_occ(world, wrap: int):
    return None if wrap else _np(world.cell_map.view(torch.uint8))


def _molmap(world) -> torch.Tensor:
    mm = world.molecule_map
    want = getattr(world, "map_dtype", torch.float32)
    if mm.dtype != want or not mm.is_contiguous():
        world.molecule_map = mm = mm.to(want).contiguous()
    return mm


# ---------------------------------------------------------------------------- placement
def free_positions(world, k: int) -> torch.Tensor:
    """Up to k distinct uniformly random free pixels (int32 (k', 2)), in random order."""
    if _is_gpu(world):
        return _hip().free_positions(world, k)
    _, _, r_lo, r_hi, _ = geom(world)
    free = torch.nonzero(~world.cell_map[r_lo:r_hi].to(torch.bool)).to(torch.int32)
    free[:, 0] += r_lo
    n = free.size(0)
    if n == 0:
        return torch.zeros(0, 2, dtype=torch.int32)
    pick = torch.randperm(n, generator=_gen_cpu)[: min(k, n)]
    return free[pick]


def divide_placement(world, idxs: torch.Tensor):
    """(parents long (k,), child positions int32 (k, 2)) for the dividing cells ``idxs``."""
    if _is_gpu(world):
        return _hip().divide_placement(world, idxs)
    pos = world.cell_positions.to(torch.int32).contiguous()
    R, C, r_lo, r_hi, wrap = geom(world)
    parents, cpos = native.host().divide_cells(
        _np(idxs.to(torch.int32)), _np(pos), R, C, r_lo, r_hi, bool(wrap), _halo_occ(world, wrap)
    )
    return torch.from_numpy(np.asarray(parents)).long(), torch.from_numpy(np.asarray(cpos))


def move_placement(world, idxs: torch.Tensor):
    """(moved long (k,), new positions int32 (k, 2))."""
    if _is_gpu(world):
        return _hip().move_placement(world, idxs)
    pos = world.cell_positions.to(torch.int32).contiguous()
    R, C, r_lo, r_hi, wrap = geom(world)
    moved, npos = native.host().move_cells(
        _np(idxs.to(torch.int32)), _np(pos), R, C, r_lo, r_hi, bool(wrap), _halo_occ(world, wrap)
    )
    return torch.from_numpy(np.asarray(moved)).long(), torch.from_numpy(np.asarray(npos))


def neighbors(world, frm: torch.Tensor, to: torch.Tensor, pos: torch.Tensor | None = None) -> torch.Tensor:
    """Unique (a < b) neighbour pairs, int32 (k, 2). ``pos`` defaults to the world's cell
    positions (a domain-decomposed world appends ghost cells of its neighbours)."""
    if _is_gpu(world):
        n = None if pos is None else int(pos.size(0))
        return _hip().neighbors(world, frm, to, pos=pos, n=n)
    if pos is None:
        pos = world.cell_positions
    pos = pos.to(torch.int32).contiguous()
    R, C, _, _, wrap = geom(world)
    out = native.host().get_neighbors(_np(frm.to(torch.int32)), _np(to.to(torch.int32)), _np(pos), R, C, bool(wrap))
    return torch.from_numpy(np.asarray(out))


def random_labels(world, k: int, length: int):
    """k random labels over [A-Za-z0-9] as packed (bytes (k, length), lengths)."""
    dev = world.__dict__["_molmap"].device
    if dev.type == "cuda":
        idx = torch.randint(0, 62, (k, length), device=dev)
    else:
        idx = torch.randint(0, 62, (k, length), generator=_gen_cpu)
    rows = _LABEL_ALPHABET.to(dev)[idx]
    return rows, torch.full((k,), length, dtype=torch.int32, device=dev)


# ---------------------------------------------------------------------------- cell <-> map exchange
def pickup_molecules(world, new: torch.Tensor, pos: torch.Tensor) -> None:
    """New cells take half of their pixel's molecules."""
    if world.__dict__["_molmap"].is_cuda:
        # pending degradation / correction: handled by the kernel path (hip_ops.map_for_pixels)
        return _hip().pickup_molecules(world, new)
    mm = _molmap(world)
    xs, ys = pos[:, 0].long(), pos[:, 1].long()
    half = mm[:, xs, ys] * 0.5
    world.cell_molecules[new] += half.T
    mm[:, xs, ys] -= half


def spill_and_free(world, idxs: torch.Tensor) -> None:
    """Killed cells release their pixel and spill their molecules onto it."""
    if world.__dict__["_molmap"].is_cuda:
        return _hip().spill_and_free(world, idxs)
    mm = _molmap(world)
    pos = world.cell_positions[idxs].long()
    xs, ys = pos[:, 0], pos[:, 1]
    world.cell_map[xs, ys] = False
    mm[:, xs, ys] += world.cell_molecules[idxs].T


def spill_and_free_mask(world, dead: torch.Tensor) -> None:
    """Cells flagged in ``dead`` (bool (n,)) spill their molecules and release their pixels."""
    if world.__dict__["_molmap"].is_cuda:
        return _hip().spill_and_free_mask(world, dead)
    spill_and_free(world, torch.nonzero(dead).flatten())


def split_cells(world, parents: torch.Tensor, children: torch.Tensor) -> None:
    """Molecules split evenly, divisions + 1 and lifetime 0 for both descendants."""
    if _is_gpu(world):
        return _hip().split_cells(world, parents, children)
    cm = world.cell_molecules
    cm[children] = cm[parents]
    both = torch.cat([parents, children])
    cm[both] *= 0.5
    dv = world.cell_divisions
    dv[children] = dv[parents]
    dv[both] += 1
    world.cell_lifetimes[both] = 0


# ---------------------------------------------------------------------------- physics
def fused_activity(world) -> bool:
    """Whether :func:`enzymatic_activity` takes the fused device path (which can also snapshot the
    state it changes, see hip_ops.enzymatic_activity)."""
    return _is_gpu(world) and not world.kinetics._stages_overridden()


def enzymatic_activity(world, save=None) -> None:
    kin = world.kinetics
    if fused_activity(world):
        return _hip().enzymatic_activity(world, save=save)
    if save is not None:
        raise ValueError("save: fused device path only")
    mm = _molmap(world)
    pos = world.cell_positions.long()
    xs, ys = pos[:, 0], pos[:, 1]
    X0 = torch.cat([world.cell_molecules, mm[:, xs, ys].T], dim=1)
    red = _mask_reducer(world)
    X1 = kin.integrate_signals(X0) if red is None else kin.integrate_signals(X0, _reduce_mask=red)
    m = world.n_molecules
    mm[:, xs, ys] = X1[:, m:].T
    world.cell_molecules[:] = X1[:, :m]


def _mask_reducer(world):
    """Host-path hook: OR a part's iteration mask over all ranks of a domain-decomposed world."""
    hook = getattr(world, "_allreduce_flags", None)
    if hook is None:
        return None

    def reduce(mask: int) -> int:
        flags = torch.tensor([(mask >> i) & 1 for i in range(4)], dtype=torch.int32)
        hook(flags)
        return sum(1 << i for i, v in enumerate(flags.tolist()) if v)

    return reduce


def diffuse(world) -> None:
    """Stencil over the owned rows -> (global) per-molecule mass totals -> correction + clamp.
    A domain-decomposed world refreshes its halo rows first and all-reduces the totals."""
    if world.__dict__["_molmap"].is_cuda:
        # the raw buffer: a pending degradation is fused into the stencil (reading
        # `molecule_map` here would apply it in a separate pass)
        return _hip().diffuse(world)
    mm = _molmap(world)
    R, C, r_lo, r_hi, wrap = geom(world)
    halo = getattr(world, "_exchange_map_halo", None)
    if halo is not None:
        halo()
    a = [float(w[0]) for w in world._diffusion]
    b = [float(w[1]) for w in world._diffusion]
    out = torch.empty_like(mm)
    totals = native.host().diffuse_stencil(mm.numpy(), out.numpy(), a, b, [1.0] * len(a), r_lo, r_hi, bool(wrap))
    tot = torch.from_numpy(np.asarray(totals))
    reduce = getattr(world, "_allreduce_totals", None)
    if reduce is not None:
        reduce(tot)
    n_pix = float(getattr(world, "_n_pix_global", (r_hi - r_lo) * C))
    native.host().diffuse_correct(mm.numpy(), out.numpy(), tot.numpy(), n_pix, r_lo, r_hi)


def permeate(world) -> None:
    if _is_gpu(world):
        return _hip().permeate(world)
    mm = _molmap(world)
    p = torch.tensor(world._permeation, dtype=torch.float32)
    if not bool((p != 0).any()):
        return
    pos = world.cell_positions.long()
    xs, ys = pos[:, 0], pos[:, 1]
    xi = world.cell_molecules
    xe = mm[:, xs, ys].T
    d_int = xi * p
    d_ext = xe * p
    world.cell_molecules[:] = xi + (d_ext - d_int)
    mm[:, xs, ys] = (xe + (d_int - d_ext)).T


def degrade(world) -> None:
    if _is_gpu(world):
        return _hip().degrade(world)
    mm = _molmap(world)
    f = torch.tensor(world._mol_degrads, dtype=torch.float32)
    mm *= f[:, None, None]
    if world.n_cells > 0:
        world.cell_molecules[:] = world.cell_molecules * f


def health_flags(world) -> torch.Tensor:
    """int32 flags: 1 non-finite / 2 negative map value (owned rows), 4 / 8 the same for cells."""
    mm = _molmap(world)
    if mm.is_cuda:
        return _hip().health_flags(world)
    _, _, r_lo, r_hi, _ = geom(world)
    own = mm[:, r_lo:r_hi]
    cm = world.cell_molecules
    f = 0
    f |= 1 if not bool(torch.isfinite(own).all()) else 0
    f |= 2 if bool((own < 0).any()) else 0
    f |= 4 if not bool(torch.isfinite(cm).all()) else 0
    f |= 8 if bool((cm < 0).any()) else 0
    return torch.tensor(f, dtype=torch.int32)


# ---------------------------------------------------------------------------- genomes
def translate(world, rows: torch.Tensor):
    """Dense tokens (k, P, D, 5) int32 and protein counts (k,) for the genomes of cells ``rows``."""
    arena = world._genomes
    if arena.data.is_cuda:
        return _hip().translate(world.genetics, arena, rows)
    data, lens = arena.view()
    sub = data[rows].contiguous()
    sl = lens[rows].contiguous()
    tokens, nprots = world.genetics.tables.translate_tokens(sub.numpy(), sl.numpy())
    return torch.from_numpy(np.asarray(tokens)), torch.from_numpy(np.asarray(nprots))


def point_mutations(world, rows, p: float, p_indel: float, p_del: float) -> torch.Tensor:
    """Mutate genomes in the arena in place; returns the (long) rows that were mutated."""
    arena = world._genomes
    if arena.data.is_cuda:
        return _hip().point_mutations(world, rows, p, p_indel, p_del)
    n = arena.n
    if rows is None:
        data = arena.data[:n].numpy()
        lens = arena.lens[:n].numpy()
        ids, overflow = native.host().point_mutations_arena(data, lens, p, p_indel, p_del)
        ids = torch.from_numpy(np.asarray(ids)).long()
        for i, seq in overflow:
            arena.set_strings([int(i)], [seq.decode("ascii")])
        if ids.numel():
            arena.version += 1
        return ids
    sub = arena.data[rows].contiguous()
    sl = arena.lens[rows].contiguous()
    ids, overflow = native.host().point_mutations_arena(sub.numpy(), sl.numpy(), p, p_indel, p_del)
    ids = torch.from_numpy(np.asarray(ids)).long()
    if ids.numel() == 0:
        return ids
    tgt = rows[ids]
    arena.set_rows(tgt, sub[ids], sl[ids])
    for i, seq in overflow:
        arena.set_strings([int(rows[int(i)])], [seq.decode("ascii")])
    return tgt


def recombinations(world, pairs: torch.Tensor, p: float) -> torch.Tensor:
    """Recombine neighbour pairs (k, 2); returns the long rows whose genomes changed."""
    arena = world._genomes
    if arena.data.is_cuda:
        return _hip().recombinations(world, pairs, p)
    pl = pairs.tolist()
    cells = sorted({c for pr in pl for c in pr})
    strs = dict(zip(cells, arena.to_strings(cells)))
    res = native.host().recombinations([(strs[a], strs[b]) for a, b in pl], p)
    if not res:
        return torch.zeros(0, dtype=torch.long)
    rows, seqs = [], []
    for s0, s1, i in res:
        a, b = pl[i]
        rows += [a, b]
        seqs += [s0, s1]
    # a cell can be in several recombined pairs: the last write wins, as in the reference
    last = {}
    for r, s in zip(rows, seqs):
        last[r] = s
    arena.set_strings(list(last), list(last.values()))
    return torch.tensor(list(last), dtype=torch.long)
