"""Host time of a top-up spawn in a running flagship world: a 10.8k-cell spawn_cells call (random 500
bp genomes from bench.random_genomes included) timed with the device drained before and after, and a
cProfile of the same call.

usage: python scripts/lab/spawn_host.py [k] [reps]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 10800
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(50000, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(10):
    bench.step(w, 50000, 500, atp)
w.synchronize()
ts = []
for r in range(reps):
    w.kill_cells(torch.arange(0, min(k, w.n_cells), device="cuda"))
    w.synchronize()
    t0 = time.perf_counter()
    g = bench.random_genomes(k, 500, "cuda")
    t1 = time.perf_counter()
    w.spawn_cells(g)
    t2 = time.perf_counter()
    w.synchronize()
    t3 = time.perf_counter()
    ts.append((round((t1 - t0) * 1e6), round((t2 - t1) * 1e6), round((t3 - t2) * 1e6)))
print("genomes / spawn_cells host / drain us:", ts)
w.kill_cells(torch.arange(0, min(k, w.n_cells), device="cuda"))
w.synchronize()
g = bench.random_genomes(k, 500, "cuda")
pr = cProfile.Profile()
pr.enable()
w.spawn_cells(g)
pr.disable()
w.synchronize()
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(35)
print(buf.getvalue())
