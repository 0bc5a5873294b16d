"""HBM sizing: what a world costs per pixel and per cell, and the largest config that fits a GPU.

The reference keeps everything in one process on one device and never sizes anything
(``python/magicsoup/world.py:195-204``: one (m, S, S) map, per-cell tensors grown by ``torch.cat``).
Here a config is planned for the 288 GB of HBM3E of an MI355X (BASELINE.json ``configs[4]``: fp16
maps "sized to fill 288 GB HBM per GPU across 8 GPUs"): :func:`footprint` models every device
buffer a GPU world holds, :func:`plan` inverts the model (the largest map side whose strip fits each
GPU of a decomposed world, for a cell density and genome size), and :func:`measured` walks a live
world's tensors so the model is checked against reality (``tests/test_gpu_kernels.py``; the
``hbm`` bench preset runs the planned config).

Per pixel (owned rows of a rank, plus two halo rows when decomposed):

* molecule map, ``m`` species x map dtype, twice: the stencil writes a second buffer and the two
  are swapped (``ops/hip_ops.py`` diffuse);
* occupancy map (1 B), placement claim map (int32) and cell-index map (int32, neighbour search /
  recombination pairs).

Per cell (capacity-managed buffers: up to 1.5x the live count, each with a spare of the same size
for order-preserving compactions):

* intracellular molecules (``m`` fp32), position (2 int32), lifetime and divisions (int32);
* the genome pool (one byte per nt, ragged: offsets + lengths per cell, no padding to the longest
  genome; twice the live bytes between collections) and a label row (16 B);
* the cell -> parameter-records map (int64) and the division / kill scratch of the native fast path;
* ragged parameter records (``csrc/hip/params.h``): one per protein of a cell's own proteome --
  per signal the packed N/Nf/Nb/A word (int32) and Kmr (fp32), plus Vmax/Kmf/Kmb/Ke (4 fp32) --
  not padded to the population's longest proteome; the pool holds about three times the live
  records (``Kinetics.reserve_cells``; replaced and dead cells' records are garbage until the next
  collection compacts them);
* the ops' per-cell scratch (integrator snapshots, neighbour keys, placement lists).
"""
from __future__ import annotations

import math

import torch

_ESIZE = {torch.float32: 4, torch.bfloat16: 2, torch.float16: 2, "fp32": 4, "bf16": 2, "fp16": 2}
_CAP = 1.5  # capacity growth factor of the per-cell buffers (worst case right after a growth)
_KIN_SPARE_BUDGET = 8 << 30  # bytes of spare parameter rows (models/kinetics.py _spare_rows)

GiB = float(1 << 30)
MI355X_HBM = 288e9  # bytes of HBM3E per GPU


def proteins_per_genome(genome_len: int) -> int:
    """Protein slots ``P`` (the longest proteome of the population) for random genomes of
    ``genome_len`` nt: about one protein per 16 nt at the tail of a large population's distribution
    (31 slots at 500 nt: the longest proteome among 500k random 500 nt genomes, measured on MI355X,
    profiles/r5/hbm_probe.log; SURVEY.md §2.3 measured 24 at 500 nt and 40 at 1 kbp for ~10k
    cells -- the tail grows with the population)."""
    return max(8, int(math.ceil(genome_len / 16.0)))


def proteins_mean(genome_len: int) -> float:
    """Mean proteome size of random genomes of ``genome_len`` nt: 6.9 / 16.8 / 54.7 proteins at
    500 / 1000 / 3000 nt (3000 random genomes each, this package's translation); about one protein
    per 55 nt, rounded up for the growth an evolving population shows."""
    return max(1.0, genome_len / 55.0)


def protein_slots(genome_len: int) -> int:
    """Protein dimension of the parameter storage for an evolving population of random genomes of
    ``genome_len`` nt: recombination joins fragments of genomes, so the longest proteome of a grown
    population far exceeds that of the random ones -- the flagship's storage widens from 45 to 82
    slots within 100 steps (profiles/r5/evolved_probe_500.log), a 5M-cell world's to 148 within 5
    steps (profiles/r5/hbm_widen.log) -- plus the storage's 50 % widening headroom
    (World._update_params_rows). World.reserve_cells(proteins=...) takes it up front, so a large
    world never re-allocates its parameter storage to widen it (old and new copy alive together)."""
    return 5 * proteins_per_genome(genome_len)


def footprint(map_size: int, n_molecules: int, cells: int, map_dtype=torch.float32, genome_len: int = 500,
              p_max: int | None = None, ranks: int = 1) -> dict:
    """Modelled device bytes of one rank of a GPU world (``ranks`` > 1: a strip of a
    domain-decomposed ``map_size``² world holding ``cells / ranks`` cells); ``p_max``: the protein
    dimension of the parameter storage (default :func:`protein_slots`). Returns the per-part
    breakdown and the total in bytes."""
    m = int(n_molecules)
    es = _ESIZE[map_dtype]
    rows = math.ceil(map_size / ranks) + (2 if ranks > 1 else 0)
    pix = rows * map_size
    n = int(math.ceil(cells / ranks))
    cap = int(n * _CAP)
    P = p_max if p_max is not None else protein_slots(genome_len)
    s = 2 * m
    rec_bytes = s * 8 + 16  # packed word + Kmr per signal, Vmax/Kmf/Kmb/Ke: one record per protein
    records = int(3 * n * max(proteins_mean(genome_len), 4.0)) + (1 << 16)  # (Kinetics.reserve_cells)
    parts = {
        "molecule_map": pix * m * es * 2,
        "pixel_maps": pix * (1 + 4 + 4),
        "cell_columns": cap * (m * 4 + 8 + 4 + 4) * 2,
        # the ragged pool: offsets + lengths (and spares) per cell, the bytes of the live genomes
        # (16-byte granules) with 2x room for new ones between collections
        "genome_pool": cap * (8 + 4) * 2 + max(16 << 20, 2 * n * ((int(genome_len * 1.1) + 15) // 16 * 16)),
        "label_arena": cap * (16 + 4) * 2,
        "row_maps": cap * (8 * 2 + 6 * 8 + 1),
        "kinetics_rows": records * rec_bytes,
        # per-cell scratch of the ops (ops/hip_ops.py): the integrator's two candidate snapshots
        # (5 states of s signals each) and cell lists, the speculative activity's saved state, the
        # neighbour-slot keys / event counts, the placement and division lists
        "op_scratch": n * (2 * 5 * s * 4 + 13 + 2 * m * 4 + 8 * 8 + 2 * 8 * 4 + 25),
    }
    parts["total"] = sum(parts.values())
    parts.update(map_size=map_size, ranks=ranks, cells_per_rank=n, p_max=P)
    return parts


MAX_MAP = 65280  # (a multiple of 256 below 2^16: the reference's positions are u16, rust/world.rs)
# pixels of one rank's map: every kernel addresses the map with 64-bit offsets (plane * pixels +
# pixel; the neighbour / placement pixel indices are long long), positions are int32 (x, y) pairs,
# so the bound is the 16-bit side above, not an index width (round 4 capped a rank at 2^30 pixels)
MAX_RANK_PIXELS = 1 << 40


def plan(hbm_bytes: float = MI355X_HBM, ranks: int = 8, n_molecules: int = 14, map_dtype="fp16",
         cells_per_pixel: float = 1e6 / 16384**2, genome_len: int = 500, reserve: float = 0.12,
         multiple: int = 256, max_map: int = MAX_MAP, max_rank_pixels: int = MAX_RANK_PIXELS) -> dict:
    """The largest map side ``S`` (a multiple of ``multiple``) whose per-rank share -- ``S / ranks``
    owned rows plus halos, ``cells_per_pixel * S²`` cells spread over the ranks -- fits
    ``hbm_bytes * (1 - reserve)`` on every GPU (the reserve covers the runtime, the RCCL buffers,
    the genome pipeline's scratch and allocator fragmentation), within a side of at most ``max_map``
    (16-bit positions, as in the reference; ``max_rank_pixels`` optionally caps a rank's pixels).
    Returns the config and its :func:`footprint`."""
    budget = hbm_bytes * (1.0 - reserve)

    def cost(S: int) -> float:
        rows = math.ceil(S / ranks) + (2 if ranks > 1 else 0)
        if S > max_map or rows * S > max_rank_pixels:
            return math.inf
        return footprint(S, n_molecules, int(cells_per_pixel * S * S), map_dtype, genome_len, ranks=ranks)["total"]

    lo, hi = multiple, multiple
    while cost(hi) <= budget:
        lo, hi = hi, hi * 2
    while hi - lo > multiple:
        mid = (lo + hi) // 2 // multiple * multiple
        if mid <= lo:
            break
        if cost(mid) <= budget:
            lo = mid
        else:
            hi = mid
    fp = footprint(lo, n_molecules, int(cells_per_pixel * lo * lo), map_dtype, genome_len, ranks=ranks)
    return {"map_size": lo, "cells": int(cells_per_pixel * lo * lo), "ranks": ranks, "map_dtype": str(map_dtype),
            "n_molecules": n_molecules, "budget_bytes": int(budget), "per_rank": fp,
            "fill": fp["total"] / hbm_bytes}


def measured(world) -> dict:
    """Device bytes held by a live world's own tensors (columns and spares, arenas, maps, kinetics
    storage, scratch), each storage counted once; compare with :func:`footprint`."""
    seen: set[int] = set()
    total = {"bytes": 0}

    def add(t):
        if isinstance(t, torch.Tensor) and t.is_cuda:
            st = t.untyped_storage()
            key = st.data_ptr()
            if key not in seen:
                seen.add(key)
                total["bytes"] += st.nbytes()
        elif isinstance(t, dict):
            for v in t.values():
                add(v)
        elif isinstance(t, (list, tuple)):
            for v in t:
                add(v)

    d = world.__dict__
    for k, v in d.items():
        if k in ("kinetics", "genetics", "chemistry"):
            continue
        add(v)
    for col in d.get("_cols", {}).values():
        add(col.buf)
        add(col.spare)
    for a in (d.get("_genomes"), d.get("_labels")):
        if a is not None:
            add(a.data)
            add(a.lens)
            add(a.__dict__.get("off"))
            add(a.__dict__.get("_spare"))
    sc = d.get("_hip_scratch")
    if sc is not None:
        add(getattr(sc, "bufs", {}))
    before = total["bytes"]
    mm = d.get("_molmap")
    maps = 0
    if isinstance(mm, torch.Tensor):
        maps = mm.untyped_storage().nbytes()
        tmp = getattr(sc, "bufs", {}).get("diff_tmp") if sc is not None else None
        maps += tmp.untyped_storage().nbytes() if isinstance(tmp, torch.Tensor) else 0
    kd = world.kinetics.__dict__
    for k, v in kd.items():
        add(v)
    # (kinetics: the parameter storage -- ragged records on the GPU -- with its slot map)
    return {"bytes": total["bytes"], "kinetics_bytes": total["bytes"] - before, "molecule_map_bytes": maps}
