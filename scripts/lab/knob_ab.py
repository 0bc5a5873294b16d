"""In-process A/B of a native setter on the flagship step loop: one world, warmed up, then blocks of
K steps alternate between the setter's values (ABAB...), each block timed through
World.synchronize(); medians and means per value. Drift of the evolving population hits every value
alike, unlike separate bench.py processes on fresh worlds.

    python scripts/lab/knob_ab.py set_place_tail=1,0 [--blocks 8] [--k 20] [--warmup 20] [--size 4096] [--cells 50000]
"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import native  # noqa: E402


def main():
    args = sys.argv[1:]
    knob = args.pop(0)
    opts = {"--blocks": 8, "--k": 20, "--warmup": 20, "--size": 4096, "--cells": 50000}
    while args:
        f, v = args.pop(0), args.pop(0)
        opts[f] = int(v)
    name, vals = knob.split("=")
    vals = [int(v) for v in vals.split(",")]
    if name.startswith("py:"):  # a module-level switch, e.g. py:magicsoup_amd.models.world._DEVCOUNT_OPS
        import importlib

        mod_name, attr = name[3:].rsplit(".", 1)
        mod = importlib.import_module(mod_name)

        def setter(v):
            setattr(mod, attr, type(getattr(mod, attr))(v))
    else:
        setter = getattr(native.hip(), name)
    S, N = opts["--size"], opts["--cells"]
    ms.set_seed(0)
    torch.manual_seed(0)
    bench._prime_rare_paths(CHEMISTRY, "cuda:0", torch.float32, 500)
    w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda:0", seed=0)
    w.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(opts["--warmup"]):
        bench.step(w, N, 500, atp)
    w.synchronize()
    times = {v: [] for v in vals}
    for b in range(opts["--blocks"]):
        for v in (vals if b % 2 == 0 else vals[::-1]):
            setter(v)
            w.synchronize()
            t = time.perf_counter()
            for _ in range(opts["--k"]):
                bench.step(w, N, 500, atp)
            w.synchronize()
            times[v].append((time.perf_counter() - t) / opts["--k"] * 1e3)
    setter(vals[0])
    out = {"knob": name, "cells_end": w.n_cells}
    for v in vals:
        out[f"{v}_median_ms"] = round(statistics.median(times[v]), 4)
        out[f"{v}_mean_ms"] = round(statistics.mean(times[v]), 4)
    out["blocks_ms"] = {str(v): [round(x, 4) for x in times[v]] for v in vals}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
