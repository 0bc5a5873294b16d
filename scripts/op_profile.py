"""torch.profiler table of one World op inside the flagship loop.

usage: python scripts/op_profile.py <op: recombinate|mutate|kill|divide|spawn|activity|diffuse> [map] [cells]"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

op = sys.argv[1]
S = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
N = int(sys.argv[3]) if len(sys.argv) > 3 else 50_000
w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(8):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
fns = {
    "recombinate": lambda: w.recombinate_cells(),
    "mutate": lambda: w.mutate_cells(),
    "kill": lambda: w.kill_cells(torch.randperm(w.n_cells, device="cuda")[:700]),
    "divide": lambda: w.divide_cells_t(w.cell_molecules[:, atp] > 5.0),
    "spawn": lambda: w.spawn_cells(bench.random_genomes(300, 500, "cuda")),
    "activity": lambda: w.enzymatic_activity(),
    "diffuse": lambda: w.diffuse_molecules(),
}
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(5):
        fns[op]()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=45, max_name_column_width=60))
