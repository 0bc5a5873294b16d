"""Paired in-process A/B of a module-level switch on ONE evolving bench world (plain, or a
virtual-strip DistributedWorld over RCCL with --virtual): the values take turns in blocks of
steps (2 untimed + K timed after each switch), so population drift and box noise cancel out.
Prints the median ms/step per value.

usage: python scripts/lab/inproc_ab.py module:NAME=v1,v2 [--virtual] [--map 4096] [--cells 50000]
       [--blocks 10] [--steps 10]   (values are Python literals)"""
import argparse
import ast
import importlib
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("toggle")
    ap.add_argument("--virtual", action="store_true")
    ap.add_argument("--map", type=int, default=4096)
    ap.add_argument("--cells", type=int, default=50000)
    ap.add_argument("--blocks", type=int, default=10)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    target, vals = a.toggle.split("=", 1)
    modname, attr = target.split(":")
    values = [ast.literal_eval(v) for v in vals.split(",")]
    import magicsoup_amd as ms

    mod = importlib.import_module(modname)
    if not hasattr(mod, attr):
        raise SystemExit(f"{modname} has no attribute {attr}")
    chem = bench._chemistry("wood_ljungdahl")
    atp = chem.molname_2_idx["ATP"]
    ms.set_seed(0)
    torch.manual_seed(0)
    torch.cuda.set_device(0)
    if a.virtual:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29541")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        from magicsoup_amd.parallel import DistributedWorld

        w = DistributedWorld(chemistry=chem, map_size=a.map, device="cuda:0", seed=0, strips=True)
    else:
        w = ms.World(chemistry=chem, map_size=a.map, device="cuda:0", seed=0)
    bench._prime_rare_paths(chem, "cuda:0", torch.float32, 500)
    w.spawn_cells(bench.random_genomes(a.cells, 500, "cuda:0"))
    for _ in range(20):
        bench.step(w, a.cells, 500, atp)
    res = {repr(v): [] for v in values}
    for _ in range(a.blocks):
        for v in values:
            setattr(mod, attr, v)
            for _ in range(2):
                bench.step(w, a.cells, 500, atp)
            w.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                bench.step(w, a.cells, 500, atp)
            w.synchronize()
            res[repr(v)].append((time.perf_counter() - t0) / a.steps * 1e3)
    print(json.dumps({"toggle": target, "virtual": a.virtual, "map": a.map, "cells": a.cells,
                      "ms_per_step_median": {k: round(statistics.median(x), 4) for k, x in res.items()},
                      "blocks": {k: [round(y, 3) for y in x] for k, x in res.items()}}), flush=True)
    if a.virtual:
        w.close()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
