"""Checkpoint timings of a decomposed world (the sharded save_state / load_state).

One rank per GPU (or one virtual strip on one GPU: MS_VIRTUAL_STRIPS semantics, the strip protocol
over the native RCCL communicator), a population of random genomes, a few bench steps, then:

* ``save_shards``   -- every rank writes its shard from device memory (no gather, no CPU World),
* ``assemble``      -- rank 0 writes the reference layout from the shards,
* ``load_shards``   -- every rank loads its own shard (parameters rebuilt on the device),
* ``load_reference``-- every rank reads its strip of the reference files,
* ``save_gathered`` -- the old path (gather to a CPU World on rank 0, re-translation there), with
  ``--gathered`` only (minutes at this size).

Usage (the N = 8 per-rank share of the m1 config on one GPU)::

    python performance/checkpoint_bench.py --map-size 5793 --cells 125000 --map-dtype fp16 --out /tmp/ck

The reference saves with ``World.save_state`` every 100 steps (performance/run_simulation.py:58-59).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--map-size", type=int, default=5793)
    ap.add_argument("--cells", type=int, default=125_000)
    ap.add_argument("--genome-size", type=int, default=500)
    ap.add_argument("--map-dtype", default="fp16")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default="/tmp/ms_ckpt")
    ap.add_argument("--gathered", action="store_true")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    rank = int(os.environ.get("RANK", "0"))
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", rank=rank, world_size=ws, device_id=torch.device("cuda", local))
    import bench
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld

    chem = bench._chemistry("wood_ljungdahl")
    mdt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[a.map_dtype]
    ms.set_seed(7 + rank)
    torch.manual_seed(7 + rank)
    dev = f"cuda:{local}"
    w = DistributedWorld(chemistry=chem, map_size=a.map_size, device=dev, seed=7, map_dtype=mdt, strips=True)
    n = a.cells // ws
    w.spawn_cells(bench.random_genomes(n, a.genome_size, dev))
    atp = chem.molname_2_idx["ATP"]
    for _ in range(a.steps):
        bench.step(w, n, a.genome_size, atp)
    w.synchronize()
    out = Path(a.out)
    if rank == 0 and out.exists():
        shutil.rmtree(out)
    dist.barrier()
    res = {"map_size": a.map_size, "cells": w.n_cells_global(), "ranks": ws, "map_dtype": a.map_dtype}

    def timed(name, fn):
        w.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        r = fn()
        w.synchronize()
        torch.cuda.synchronize()
        dist.barrier()
        res[name + "_s"] = round(time.perf_counter() - t0, 3)
        return r

    before = {"n": w.n_cells, "pos": w.global_positions().clone(), "mol": w.cell_molecules.clone()}
    timed("save_shards", lambda: w.save_state(out / "state", assemble=False))
    if rank == 0:
        from magicsoup_amd.utils import checkpoint

        timed_single = time.perf_counter()
        checkpoint.assemble_state(out / "state")
        res["assemble_s"] = round(time.perf_counter() - timed_single, 3)
        shutil.copytree(out / "state", out / "refonly", ignore=shutil.ignore_patterns("shards"))
    dist.barrier()
    kind = timed("load_shards", lambda: w.load_state(out / "state"))
    assert kind == "shard"
    same = w.n_cells == before["n"] and torch.equal(w.global_positions(), before["pos"]) and torch.equal(
        w.cell_molecules, before["mol"])
    kind = timed("load_reference", lambda: w.load_state(out / "refonly"))
    assert kind == "reference"
    same = same and torch.equal(w.global_positions(), before["pos"])
    res["roundtrip_exact"] = bool(same)
    if a.gathered:
        timed("save_gathered", lambda: w.save_state_gathered(out / "gathered"))
    sizes = {}
    if rank == 0:
        for p in sorted((out / "state").rglob("*")):
            if p.is_file():
                sizes[str(p.relative_to(out / "state"))] = p.stat().st_size
        res["bytes_total"] = sum(sizes.values())
        res["bytes_shards"] = sum(v for k, v in sizes.items() if k.startswith("shards"))
        print(json.dumps(res), flush=True)
    w.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
