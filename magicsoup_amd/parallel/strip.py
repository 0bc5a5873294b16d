"""Device primitives of the strip protocols (:mod:`magicsoup_amd.parallel.dist_world`).

GPU worlds run the gfx950 kernels of ``csrc/hip/dist.hip``; CPU worlds (gloo tests, rehearsals)
run the same steps as plain tensor ops. Layout of a strip: rows ``1..H`` owned, rows ``0`` and
``H + 1`` halo copies of the neighbours' boundary rows (see ``World._map_shape`` / ``_geom``).

Cell records (division children and migrants) share one byte layout on both paths::

    int32 y, genome length, label length, divisions, lifetime | float32 molecules[m]
    | label row (lw bytes) | genome row (gw bytes)

``lw`` / ``gw`` are the sender's label row width and genome length bound (multiples of 16),
announced in the header; GPU genomes are read from / written to the genome pool.
"""
from __future__ import annotations

import torch

_U8 = torch.uint8
HDR = 4  # header words: record count, label row width, genome row width, molecules


def _hip():
    from magicsoup_amd.ops.hip_ops import _m

    return _m()


def _stream() -> int:
    from magicsoup_amd.ops.hip_ops import _stream as s

    return s()


def _p(t) -> int:
    return 0 if t is None else t.data_ptr()


def record_bytes(m: int, lw: int, gw: int) -> int:
    return 4 * (5 + m) + lw + gw


def _cmap(world) -> torch.Tensor:
    return world.cell_map.view(_U8)


# ---------------------------------------------------------------------------- division: marks
def marks(world, cells: torch.Tensor | None, up: torch.Tensor, dn: torch.Tensor, mask: torch.Tensor | None = None) -> None:
    """Bytes per column of the owned boundary rows into ``up`` (row 1) / ``dn`` (row H): 1 occupied,
    3 occupied by one of the dividing ``cells`` (or, GPU, the cells selected by ``mask``)."""
    H, C = world.H, world.map_size
    cm = _cmap(world)
    if cm.is_cuda:
        if mask is not None:
            _hip().strip_marks(C, H, _p(cm), int(mask.numel()), 0, _p(mask), _p(world.cell_positions), _p(up), _p(dn),
                               _stream())
        else:
            _hip().strip_marks(C, H, _p(cm), int(cells.numel()), _p(cells), 0, _p(world.cell_positions), _p(up),
                               _p(dn), _stream())
        return
    up.copy_((cm[1] != 0).to(_U8))
    dn.copy_((cm[H] != 0).to(_U8))
    if cells.numel():
        p = world.cell_positions[cells].long()
        up[p[p[:, 0] == 1, 1]] = 3
        dn[p[p[:, 0] == H, 1]] = 3


def reserve(world, from_up: torch.Tensor, from_dn: torch.Tensor) -> None:
    """Halo occupancy from the neighbours' marks; owned boundary pixels next to a neighbour's
    dividing cell reserved (2) for that neighbour's claims.

    Known statistical deviation from a single map (documented in docs/architecture.md): the
    reference places all children in one random priority order over the whole population
    (rust/world.rs:59-97). Here a reserved pixel is closed to the owning rank's own dividing cells
    even when the neighbour's cell ends up claiming a different pixel, so next to a strip boundary
    children favour the neighbour's side. The effect is confined to the two boundary rows per strip
    and keeps the protocol free of an accept / reject round trip."""
    H, C = world.H, world.map_size
    cm = _cmap(world)
    if cm.is_cuda:
        _hip().strip_reserve(C, H, _p(from_up), _p(from_dn), _p(cm), _stream())
        return
    cm[0] = from_up & 1
    cm[H + 1] = from_dn & 1
    for row, src in ((1, from_up), (H, from_dn)):
        d = (src & 2) != 0
        near = d | torch.roll(d, 1) | torch.roll(d, -1)
        r = cm[row]
        r[(r == 0) & near] = 2


def clear(world) -> None:
    """Halo rows empty again, reservations released."""
    H, C = world.H, world.map_size
    cm = _cmap(world)
    if cm.is_cuda:
        _hip().strip_clear(C, H, _p(cm), _stream())
        return
    cm[0] = 0
    cm[H + 1] = 0
    for row in (1, H):
        r = cm[row]
        r[r == 2] = 0


# ---------------------------------------------------------------------------- division: winners
def split_winners_gpu(world, cells: torch.Tensor | None, result: torch.Tensor, par: torch.Tensor, npos: torch.Tensor,
                      status: torch.Tensor) -> None:
    """Placement results (pixel or -1 per dividing cell) -> per class (local, up, down) the winners'
    cells ``par[c * k:]`` and pixels ``npos[c * k:]`` in list order; counts into ``status[0:3]`` and
    the outgoing headers' counts into ``status[4]`` (to up) / ``status[8]`` (to down)."""
    k = int(cells.numel()) if cells is not None else int(result.numel())
    _hip().place_split(k, _p(result), _p(cells), world.map_size, world.H, _p(par), _p(npos), _p(status),
                       _p(status[4:]), _p(status[8:]), int(world._labels.width), int(world._genomes.width),
                       world.n_molecules, _stream())


def split_winners_cpu(world, parents: torch.Tensor, cpos: torch.Tensor):
    """(local, up, down) index tensors into ``parents`` / ``cpos`` by destination row."""
    x = cpos[:, 0]
    up = torch.nonzero(x == 0).flatten()
    dn = torch.nonzero(x == world.H + 1).flatten()
    loc = torch.nonzero((x != 0) & (x != world.H + 1)).flatten()
    return loc, up, dn


# ---------------------------------------------------------------------------- records
def pack(world, par_up, pos_up, par_dn, pos_dn, child: bool, out_up: torch.Tensor | None, out_dn: torch.Tensor | None):
    """Records of cells ``par_*`` (their children when ``child``) landing on columns ``pos_*[:, 1]``
    into the uint8 buffers ``out_*`` (k x record_bytes)."""
    k_up = 0 if par_up is None else int(par_up.numel())
    k_dn = 0 if par_dn is None else int(par_dn.numel())
    if k_up + k_dn == 0:
        return
    g, lab = world._genomes, world._labels
    m = world.n_molecules
    if world.cell_molecules.is_cuda:
        _hip().rec_pack(k_up, k_dn, _p(par_up), _p(pos_up), _p(par_dn), _p(pos_dn), _p(world.cell_molecules),
                        _p(world.cell_positions), _p(world.cell_lifetimes), _p(world.cell_divisions), g.args(),
                        _p(g.lens), int(g.width), _p(lab.data), _p(lab.lens), int(lab.width), m, bool(child),
                        _p(out_up), _p(out_dn), _stream())
        return
    for cells, pos, out in ((par_up, pos_up, out_up), (par_dn, pos_dn, out_dn)):
        k = 0 if cells is None else int(cells.numel())
        if k == 0:
            continue
        mol = world.cell_molecules[cells].to(torch.float32)
        div = world.cell_divisions[cells].to(torch.int32)
        life = world.cell_lifetimes[cells].to(torch.int32)
        if child:
            mol, div, life = mol * 0.5, div + 1, torch.zeros_like(life)
        head = torch.stack([pos[:, 1].to(torch.int32), g.lens[cells], lab.lens[cells], div, life], dim=1)
        cols = [head.contiguous().view(_U8).reshape(k, -1), mol.contiguous().view(_U8).reshape(k, -1),
                lab.data[cells].reshape(k, -1), g.data[cells].reshape(k, -1)]
        out.copy_(torch.cat(cols, dim=1).reshape(out.shape))


def unpack(world, n0: int, buf_up, hdr_up, buf_dn, hdr_dn) -> None:
    """Write the records from the upper neighbour (onto row 1) and from the lower one (row H) as
    rows n0, n0 + 1, ... of every per-cell array (already grown) and claim their pixels."""
    k_up, k_dn = int(hdr_up[0]), int(hdr_dn[0])
    if k_up + k_dn == 0:
        return
    g, lab = world._genomes, world._labels
    m, H, C = world.n_molecules, world.H, world.map_size
    if world.cell_molecules.is_cuda:
        # (the genomes go to fresh space of the genome pool)
        need = k_up * ((int(hdr_up[2]) + 15) // 16 * 16) + k_dn * ((int(hdr_dn[2]) + 15) // 16 * 16)
        g.ensure(need)
        g.top_ub += need
        _hip().rec_unpack(n0, k_up, _p(buf_up), int(hdr_up[1]), int(hdr_up[2]), k_dn, _p(buf_dn), int(hdr_dn[1]),
                          int(hdr_dn[2]), C, H, _p(world.cell_molecules), _p(world.cell_positions),
                          _p(world.cell_lifetimes), _p(world.cell_divisions), g.args(), _p(g.lens),
                          max(int(hdr_up[2]), int(hdr_dn[2])),
                          _p(lab.data), _p(lab.lens), int(lab.width), m, _p(_cmap(world)), _stream())
        return
    cm = _cmap(world)
    row0 = n0
    for buf, hdr, x in ((buf_up, hdr_up, 1), (buf_dn, hdr_dn, H)):
        k = int(hdr[0])
        if k == 0:
            continue
        lw, gw = int(hdr[1]), int(hdr[2])
        recs = buf.view(k, record_bytes(m, lw, gw))
        head = recs[:, :20].contiguous().view(torch.int32).reshape(k, 5)
        mol = recs[:, 20 : 20 + 4 * m].contiguous().view(torch.float32).reshape(k, m)
        ldat = recs[:, 20 + 4 * m : 20 + 4 * m + lw]
        gdat = recs[:, 20 + 4 * m + lw :]
        rows = torch.arange(row0, row0 + k)
        ys = head[:, 0]
        world.cell_positions[rows] = torch.stack([torch.full_like(ys, x), ys], dim=1)
        world.cell_molecules[rows] = mol
        world.cell_divisions[rows] = head[:, 3]
        world.cell_lifetimes[rows] = head[:, 4]
        glen = head[:, 1].clamp(max=g.width)
        llen = head[:, 2].clamp(max=lab.width)
        w = min(gw, g.width)
        g.data[rows] = 0
        g.data[rows, :w] = gdat[:, :w]
        g.lens[rows] = glen
        w = min(lw, lab.width)
        lab.data[rows] = 0
        lab.data[rows, :w] = ldat[:, :w]
        lab.lens[rows] = llen
        cm[x, ys.long()] = 1
        row0 += k


# ---------------------------------------------------------------------------- diffusion halo
def halo_pack(world, send_up: torch.Tensor, send_dn: torch.Tensor) -> None:
    mm = world.__dict__["_molmap"]
    H = world.H
    if mm.is_cuda:
        _hip().halo_pack(int(mm.size(0)), world.map_size, H, mm.element_size(), _p(mm), _p(send_up), _p(send_dn),
                         _stream())
        return
    m = int(mm.size(0))
    send_up.view(m, -1).copy_(mm[:, 1])
    send_dn.view(m, -1).copy_(mm[:, H])


def halo_unpack(world, from_up: torch.Tensor, from_dn: torch.Tensor) -> None:
    mm = world.__dict__["_molmap"]
    H = world.H
    if mm.is_cuda:
        _hip().halo_unpack(int(mm.size(0)), world.map_size, H, mm.element_size(), _p(mm), _p(from_up), _p(from_dn),
                           _stream())
        return
    m = int(mm.size(0))
    mm[:, 0].copy_(from_up.view(m, -1))
    mm[:, H + 1].copy_(from_dn.view(m, -1))
