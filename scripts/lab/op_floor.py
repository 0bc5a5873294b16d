"""Per-call cost of each World op on a small population (the launch / host floor a rank of a
multi-GPU job pays): wall time of one call with the device drained before and after (``sync``),
and the host time until the call returns (``issue``, no drain after).

usage: python scripts/lab/op_floor.py [map_size] [cells] [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1448
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6250
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(10):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()


def none_mask():
    return torch.zeros(w.n_cells, dtype=torch.bool, device="cuda")


def few_mask(k=50):
    m = torch.zeros(w.n_cells, dtype=torch.bool, device="cuda")
    m[torch.randperm(w.n_cells, device="cuda")[:k]] = True
    return m


cases = {
    "enzymatic_activity": (lambda: None, lambda _: w.enzymatic_activity()),
    "kill_cells(mask, none)": (none_mask, lambda m: w.kill_cells(m)),
    "divide_cells_t(mask, none)": (none_mask, lambda m: w.divide_cells_t(m)),
    "divide_cells_t(mask, 50)": (few_mask, lambda m: w.divide_cells_t(m)),
    "kill_cells(mask, 50)": (few_mask, lambda m: w.kill_cells(m)),
    "recombinate_cells()": (lambda: None, lambda _: w.recombinate_cells()),
    "mutate_cells()": (lambda: None, lambda _: w.mutate_cells()),
    "degrade_molecules": (lambda: None, lambda _: w.degrade_molecules()),
    "diffuse_molecules": (lambda: None, lambda _: w.diffuse_molecules()),
    "increment_cell_lifetimes": (lambda: None, lambda _: w.increment_cell_lifetimes()),
    "spawn_cells(50)": (lambda: bench.random_genomes(50, 500, "cuda"), lambda g: w.spawn_cells(g)),
}
print(f"{S}^2 map, {w.n_cells} cells, {reps} reps: median us per call")
print(f"{'op':30s} {'sync':>8s} {'issue':>8s}")
for name, (prep, fn) in cases.items():
    t_sync, t_issue = [], []
    for _ in range(reps):
        arg = prep()
        w._reconcile()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(arg)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t_issue.append((t1 - t0) * 1e6)
        t_sync.append((t2 - t0) * 1e6)
        if w.n_cells < N // 2 or w.n_cells > 2 * N:
            bench.step(w, N, 500, atp)
    print(f"{name:30s} {statistics.median(t_sync):8.1f} {statistics.median(t_issue):8.1f}")
