"""Paired A/B of the early diffusion stencil and of the eager genome chains on ONE evolving flagship world: the variants take turns
in blocks of steps (2 untimed + K timed after each switch), so population drift and box-to-box noise
cancel out. Prints the median ms/step of each variant.

usage: python scripts/lab/early_ab.py [map_size] [cells] [blocks] [steps_per_block]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.models import world as world_mod  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
blocks = int(sys.argv[3]) if len(sys.argv) > 3 else 6
K = int(sys.argv[4]) if len(sys.argv) > 4 else 10
chem = bench._chemistry("wood_ljungdahl")
atp = chem.molname_2_idx["ATP"]
ms.set_seed(0)
torch.manual_seed(0)
w = ms.World(chemistry=chem, map_size=S, device="cuda:0", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
for _ in range(20):
    bench.step(w, N, 500, atp)
# (early diffusion, flush at once when it is pending, where the kill issues it, eager chains + lazy join)
VARIANTS = {"off": (False, True, "spill", True), "off_join_at_diffuse": (False, True, "spill", False),
            "spill_flush": (True, True, "spill", True), "synced_flush": (True, True, "synced", True)}
if os.environ.get("AB_OLD"):
    VARIANTS = {"off": (False, True, "spill", False), "spill_flush": (True, True, "spill", False),
                "spill_late": (True, False, "spill", False), "synced_flush": (True, True, "synced", False)}
res = {k: [] for k in VARIANTS}
for b in range(blocks):
    for name, (early, flush, at, chains) in VARIANTS.items():
        w.__dict__["_early_diffuse"] = early
        w.__dict__["_early_chains"] = chains
        world_mod._FLUSH_EARLY = flush
        hip_ops.EARLY_DIFFUSE_AT = at
        for _ in range(2):
            bench.step(w, N, 500, atp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            bench.step(w, N, 500, atp)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / K * 1e3)
print(json.dumps({"map": S, "cells": N, "ms_per_step_median": {k: round(statistics.median(v), 4) for k, v in res.items()},
                  "blocks": {k: [round(x, 3) for x in v] for k, v in res.items()}}))
