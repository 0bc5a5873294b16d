"""cProfile of repeated calls of one World op on a small GPU population (host-side cost breakdown).

usage: python scripts/op_cprofile.py <op: recombinate|mutate|kill|kill50|divide|divide50|activity|spawn|diffuse> [reps]
    [cells]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

op = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
w = ms.World(chemistry=CHEMISTRY, map_size=1448, device="cuda", seed=0)
ncell = int(sys.argv[3]) if len(sys.argv) > 3 else 6250
w.spawn_cells(bench.random_genomes(ncell, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(10):
    bench.step(w, ncell, 500, atp)
torch.cuda.synchronize()
few = torch.zeros(w.n_cells, dtype=torch.bool, device="cuda")
fns = {
    "recombinate": lambda: w.recombinate_cells(),
    "mutate": lambda: w.mutate_cells(),
    "kill": lambda: w.kill_cells(torch.zeros(w.n_cells, dtype=torch.bool, device="cuda")),
    "divide": lambda: w.divide_cells_t(torch.zeros(w.n_cells, dtype=torch.bool, device="cuda")),
    "divide50": lambda: w.divide_cells_t(torch.rand(w.n_cells, device="cuda") < 50 / w.n_cells),
    "kill50": lambda: w.kill_cells(torch.rand(w.n_cells, device="cuda") < 50 / w.n_cells),
    "activity": lambda: w.enzymatic_activity(),
    "spawn": lambda: w.spawn_cells(bench.random_genomes(20, 500, "cuda")),
    "diffuse": lambda: w.diffuse_molecules(),
}
fn = fns[op]
for _ in range(20):
    fn()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(reps):
    fn()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(35)
