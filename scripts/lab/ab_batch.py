"""In-process A/B of the graph batching of native launches (csrc/hip/launch.h): one world steps
through alternating blocks of bench steps with batching on and off (set_graph_batch at run time), so
box and process variance cancel; prints the median ms/step of each setting.

usage: python scripts/lab/ab_batch.py [map_size] [cells] [blocks] [steps_per_block]
MS_VIRTUAL_STRIPS=1: a one-rank DistributedWorld running the strip protocol (RCCL to itself)."""
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

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1448
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6250
blocks = int(sys.argv[3]) if len(sys.argv) > 3 else 10
per = int(sys.argv[4]) if len(sys.argv) > 4 else 20
virtual = os.environ.get("MS_VIRTUAL_STRIPS") == "1"
if virtual:
    import torch.distributed as dist

    from magicsoup_amd.parallel import DistributedWorld

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29548")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    w = DistributedWorld(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0, strips=True)
else:
    w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
m = native.hip()
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(20):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
res = {True: [], False: []}
for b in range(blocks):
    for on in ((True, False) if b % 2 == 0 else (False, True)):
        m.set_graph_batch(on)
        bench.step(w, N, 500, atp)  # (one untimed step in the new setting)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(per):
            bench.step(w, N, 500, atp)
        torch.cuda.synchronize()
        res[on].append((time.perf_counter() - t0) / per * 1e3)
m.set_graph_batch(False)
print(json.dumps({"map": S, "cells": N, "virtual": virtual, "batched_ms": round(statistics.median(res[True]), 4),
                  "direct_ms": round(statistics.median(res[False]), 4),
                  "batched_blocks": [round(x, 3) for x in res[True]], "direct_blocks": [round(x, 3) for x in res[False]]}))
