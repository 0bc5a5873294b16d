"""Evolved-population probe: run the flagship loop (bench.step) for many steps and report, every
``--every`` steps, the mean step time of the last block of steps, the active-protein / non-zero
distribution of the population and the time of one enzymatic_activity on that state.

    python scripts/lab/evolved_probe.py [--steps 500] [--every 50] [--map-size 4096] [--cells 50000]
        [--modes 128]

The reference's macro benchmark runs 200 steps of an evolving population
(``performance/run_simulation.py:120``); a freshly spawned population (the first few dozen steps)
has small proteomes, a grown one does not.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import native  # noqa: E402


def population_stats(w) -> dict:
    kin = w.kinetics
    vmax = kin.Vmax
    na = (~(vmax <= 0)).sum(1)
    N = kin.N
    act = ~(vmax <= 0)
    nz = ((N != 0) | (kin.A != 0)).sum(2) * act  # non-zero signals per active protein
    nzmax = nz.amax(1)
    out = {
        "cells": int(w.n_cells),
        "P": int(N.size(1)),
        "na_mean": round(float(na.float().mean()), 2),
        "na_p50": int(na.float().quantile(0.5)),
        "na_p99": int(na.float().quantile(0.99)),
        "na_max": int(na.max()),
        "na_gt32": int((na > 32).sum()),
        "na_gt64": int((na > 64).sum()),
        "nz_gt16": int((nzmax > 16).sum()),
        "nz_gt32": int((nzmax > 32).sum()),
        "genome_mean": round(float(w._genomes.lens[: w.n_cells].float().mean()), 1),
    }
    return out


def timed_activity(w, iters: int = 5) -> float:
    from magicsoup_amd.ops import hip_ops

    buf = hip_ops.save_cell_state(w)
    w.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        hip_ops.restore_cell_state(w, buf)
        w.synchronize()
        a.record()
        w.enzymatic_activity()
        b.record()
        w.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    hip_ops.restore_cell_state(w, buf)
    w.synchronize()
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--every", type=int, default=50)
    ap.add_argument("--map-size", type=int, default=4096)
    ap.add_argument("--cells", type=int, default=50_000)
    ap.add_argument("--modes", default="", help="comma-separated integrator modes to time as well")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    ms.set_seed(a.seed)
    torch.manual_seed(a.seed)
    dev = "cuda:0"
    bench._prime_rare_paths(CHEMISTRY, dev, torch.float32, 500)
    w = ms.World(chemistry=CHEMISTRY, map_size=a.map_size, device=dev, seed=a.seed)
    w.spawn_cells(bench.random_genomes(a.cells, 500, dev))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    w.synchronize()
    t0 = time.perf_counter()
    done = 0
    while done < a.steps:
        k = min(a.every, a.steps - done)
        t1 = time.perf_counter()
        for _ in range(k):
            bench.step(w, a.cells, 500, atp)
        w.synchronize()
        dt = (time.perf_counter() - t1) / k * 1e3
        done += k
        rec = {"step": done, "ms_per_step": round(dt, 4)}
        rec.update(population_stats(w))
        rec["us_activity"] = timed_activity(w)
        for mode in [int(x) for x in a.modes.split(",") if x]:  # integrator launch modes (A/B)
            native.hip().set_integrate_mode(mode)
            rec[f"us_activity_mode{mode}"] = timed_activity(w)
        if a.modes:
            native.hip().set_integrate_mode(0)
        print(json.dumps(rec), flush=True)
    w.synchronize()
    print(json.dumps({"total_s": round(time.perf_counter() - t0, 2), "steps": a.steps}), flush=True)


if __name__ == "__main__":
    main()
