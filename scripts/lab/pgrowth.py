"""Growth of the kinetics protein bound (Kinetics._P) against the population's longest proteome and
genome over a long evolving flagship run.

usage: python scripts/lab/pgrowth.py [steps] [every]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
every = int(sys.argv[2]) if len(sys.argv) > 2 else 100
S, N = (int(x) for x in (sys.argv[3], sys.argv[4])) if len(sys.argv) > 4 else (4096, 50000)
w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for i in range(steps):
    try:
        bench.step(w, N, 500, atp)
    except RuntimeError as e:
        print("step", i, "failed:", e, flush=True)
        break
    if i % every == 0 or i == steps - 1:
        w.synchronize()
        kin = w.kinetics
        slot = kin._slot_tensor()
        cnt = (slot >> 32) & ((1 << 16) - 1)
        lens = w._genomes.lens[: w.n_cells]
        print({"step": i, "cells": w.n_cells, "P": kin._P(), "max_proteome": int(cnt.max()),
               "mean_proteome": round(float(cnt.float().mean()), 1), "max_genome": int(lens.max()),
               "mean_genome": round(float(lens.float().mean()), 1)}, flush=True)
