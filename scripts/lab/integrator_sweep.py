"""enzymatic_activity time against the cell count on the flagship map (4096^2, WL, 500 bp): a
step-shaped curve would mean the integrator launch is quantised by the cells resident per round.
usage: python scripts/lab/integrator_sweep.py [n ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [24_000, 30_000, 36_000, 40_000, 45_000, 48_000, 50_000, 52_000, 56_000,
                                           60_000]
for n in sizes:
    w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(n, 500, "cuda"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(3):
        bench.step(w, n, 500, atp)
    w.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w.enzymatic_activity()
    w.synchronize()
    a.record()
    for _ in range(20):
        w.enzymatic_activity()
    b.record()
    w.synchronize()
    print(f"cells {w.n_cells:6d}  enzymatic_activity {a.elapsed_time(b) / 20 * 1e3:7.1f} us", flush=True)
    del w
    torch.cuda.empty_cache()
