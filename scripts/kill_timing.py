"""Host-side timing of the kill_cells GPU path, piece by piece (each piece synchronised)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops, world_ops  # noqa: E402

w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(50000, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(5):
    bench.step(w, 50000, 500, atp)
torch.cuda.synchronize()
T = {}


def tm(name, fn, reps=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    T[name] = (time.perf_counter() - t0) / reps * 1e6
    return out


n = w.n_cells
dead = torch.rand(n, device="cuda") < 0.01
tm("empty_sync", lambda: torch.cuda.synchronize())
tm("select_rest", lambda: hip_ops.select(dead, "clear", rest=True))
tm("select", lambda: hip_ops.select(dead, "clear"))
keep_idx, dead_idx, _ = hip_ops.select(dead, "clear", rest=True)


def compact_pairs():
    pairs = [(col.view(n), col.spare_rows(int(keep_idx.numel()))) for col in w._cols.values()]
    pairs += w._genomes.compact_pairs(int(keep_idx.numel())) + w._labels.compact_pairs(int(keep_idx.numel()))
    return pairs


pairs = tm("build_pairs", compact_pairs)
tm("gather_rows", lambda: hip_ops.gather_rows(pairs, int(keep_idx.numel()), src_rows=keep_idx))
tm("kill_cells_full", lambda: (w.kill_cells(torch.zeros(w.n_cells, dtype=torch.bool, device="cuda"))), reps=20)
t0 = time.perf_counter()
for _ in range(20):
    w.kill_cells(torch.rand(w.n_cells, device="cuda") < 0.002)
    w.spawn_cells(bench.random_genomes(100, 500, "cuda"))
torch.cuda.synchronize()
T["kill+spawn100"] = (time.perf_counter() - t0) / 20 * 1e6
for k, v in T.items():
    print(f"{k:20s} {v:8.1f} us")
