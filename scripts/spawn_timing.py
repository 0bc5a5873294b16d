"""Where does spawn_cells spend its time on the GPU? (cProfile over repeated small spawns)"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(50000, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(5):
    bench.step(w, 50000, 500, atp)
torch.cuda.synchronize()
g = [bench.random_genomes(100, 500, "cuda") for _ in range(20)]
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for i in range(20):
    w.spawn_cells(g[i])
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(35)
