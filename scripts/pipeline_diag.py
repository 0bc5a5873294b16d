"""Device genome pipeline diagnostics on the flagship bench world: which flags the pending calls
raise per step, how long reconcile blocks the host, and the step rate with / without the pipeline.

usage: python scripts/pipeline_diag.py [--map-size 4096 --cells 50000 --steps 30]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.ops import genome_pipeline as gp  # noqa: E402


def run(a, sync_path: bool) -> dict:
    if sync_path:
        os.environ["MS_SYNC_GENETICS"] = "1"
    else:
        os.environ.pop("MS_SYNC_GENETICS", None)
    chem = bench._chemistry("wl")
    atp = chem.molname_2_idx["ATP"]
    ms.set_seed(1)
    torch.manual_seed(1)
    w = ms.World(chemistry=chem, map_size=a.map_size, device="cuda", seed=1)
    w.spawn_cells(bench.random_genomes(a.cells, 500, "cuda"))
    flags = collections.Counter()
    block = []
    orig = gp.reconcile

    def rec(world):
        st = world.__dict__.get("_gp_state")
        if st and st["pending"]:
            t = time.perf_counter()
            st["pending"][-1].event.synchronize()
            block.append(time.perf_counter() - t)
            for pd in st["pending"]:
                flags[(pd.kind, int(pd.host[1]))] += 1
        orig(world)

    gp.reconcile = rec
    try:
        for _ in range(5):
            bench.step(w, a.cells, 500, atp)
        torch.cuda.synchronize()
        flags.clear()
        block.clear()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            bench.step(w, a.cells, 500, atp)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    finally:
        gp.reconcile = orig
    return {
        "path": "sync" if sync_path else "pipeline",
        "steps_per_s": round(a.steps / dt, 1),
        "flags": {f"{k}:{v}": c for (k, v), c in sorted(flags.items())},
        "reconcile_wait_us_mean": round(1e6 * sum(block) / max(len(block), 1), 1),
        "arena_width": int(w._genomes.width),
        "P": int(w.kinetics._P()),
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--map-size", type=int, default=4096)
    p.add_argument("--cells", type=int, default=50000)
    p.add_argument("--steps", type=int, default=30)
    a = p.parse_args()
    for sync_path in (False, True, False, True):
        print(json.dumps(run(a, sync_path)), flush=True)


if __name__ == "__main__":
    main()
