"""Host-side profile (cProfile) of the flagship step; prints the top functions by cumulative time."""
import cProfile
import pstats
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

map_size = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cells = int(sys.argv[2]) if len(sys.argv) > 2 else 40000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = "cuda" if torch.cuda.is_available() else "cpu"
w = ms.World(chemistry=CHEMISTRY, map_size=map_size, device=dev, seed=0)
w.spawn_cells(bench.random_genomes(cells, 500, dev))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(3):
    bench.step(w, cells, 500, atp)
torch.cuda.synchronize() if dev == "cuda" else None
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    bench.step(w, cells, 500, atp)
torch.cuda.synchronize() if dev == "cuda" else None
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("cumulative").print_stats(45)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("tottime").print_stats(30)
