"""Driver for PMC passes over the integrator: a flagship-like state after a few bench steps, then
`reps` enzymatic_activity calls with the speculative all-parts launch (mode 0) followed by `reps`
with the per-part register launches (mode 128); kernel names tell the two apart.

usage: python scripts/lab/integrator_pmc.py [map_size] [cells] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import native  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cells = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(5):
    bench.step(w, cells, 500, atp)
torch.cuda.synchronize()
for mode in (0, 128):  # speculative all-parts launch, per-part register launches
    native.hip().set_integrate_mode(mode)
    for _ in range(reps):
        w.enzymatic_activity()
    torch.cuda.synchronize()
print("done", w.n_cells)
