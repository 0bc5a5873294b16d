"""Host time of each statement of the flagship step between the kill's read-back and the stencil
launch (where the compute queue idles while the host issues the next launches): perf_counter_ns
marks around the bench loop's statements, means over the timed steps.
usage: python scripts/lab/glue_timeline.py [map_size] [cells] [steps]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
atp = CHEMISTRY.molname_2_idx["ATP"]
w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
bench._prime_rare_paths(CHEMISTRY, "cuda", torch.float32, 500)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
for _ in range(20):
    bench.step(w, N, 500, atp)
w.synchronize()
acc = collections.defaultdict(float)
ns = time.perf_counter_ns
for _ in range(steps):
    t = [ns()]
    n = w.n_cells
    dilute = bench._dilution_mask(n, max(1, n - N), "cuda") if n > N else None
    t.append(ns())
    w.enzymatic_activity()
    t.append(ns())
    kill = w.cell_molecules[:, atp] < 1.0
    if dilute is not None:
        kill |= dilute
    t.append(ns())
    w.kill_cells(kill)
    t.append(ns())
    nk = w.n_cells
    t.append(ns())
    repl = w.cell_molecules[:, atp] > 5.0
    t.append(ns())
    w.cell_molecules[:, atp] -= 4.0 * repl
    t.append(ns())
    w.divide_cells_t(repl, lazy=True)
    t.append(ns())
    w.recombinate_cells()
    w.mutate_cells()
    t.append(ns())
    w.degrade_molecules()
    t.append(ns())
    w.diffuse_molecules()
    t.append(ns())
    w.increment_cell_lifetimes()
    t.append(ns())
    names = ["top+dilute", "activity", "kill masks", "kill_cells (incl. wait)", "n_cells", "repl mask",
             "atp -= 4", "divide_cells_t", "rec+mut (queued)", "degrade", "diffuse (+flush)", "lifetimes"]
    for i, nm in enumerate(names):
        acc[nm] += (t[i + 1] - t[i]) / 1e3
torch.cuda.synchronize()
for nm, v in acc.items():
    print(f"{nm:26s} {v / steps:8.1f} us", flush=True)
