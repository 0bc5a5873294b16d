"""Host time between a select read-back and the next launch of the op (kill / divide paths), measured
with perf_counter on the flagship bench world without a profiler attached.

usage: python scripts/lab/host_gaps.py [steps]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
chem = bench._chemistry("wl")
atp = chem.molname_2_idx["ATP"]
w = ms.World(chemistry=chem, map_size=4096, device="cuda", seed=1)
w.spawn_cells(bench.random_genomes(50000, 500, "cuda"))
for _ in range(5):
    bench.step(w, 50000, 500, atp)
torch.cuda.synchronize()

acc = collections.defaultdict(float)
cnt = collections.Counter()
last = {"t": None}
orig_select, orig_gather = hip_ops.select, hip_ops.gather_rows


def sel(*a, **k):
    t0 = time.perf_counter()
    r = orig_select(*a, **k)
    t1 = time.perf_counter()
    acc["select (incl. wait)"] += t1 - t0
    cnt["select (incl. wait)"] += 1
    last["t"] = t1
    return r


def gat(*a, **k):
    if last["t"] is not None:
        acc["select -> gather_rows"] += time.perf_counter() - last["t"]
        cnt["select -> gather_rows"] += 1
        last["t"] = None
    t0 = time.perf_counter()
    r = orig_gather(*a, **k)
    acc["gather_rows call"] += time.perf_counter() - t0
    cnt["gather_rows call"] += 1
    return r


hip_ops.select, hip_ops.gather_rows = sel, gat
ops = collections.defaultdict(float)
for name in ("kill_cells", "divide_cells_t", "spawn_cells", "enzymatic_activity", "recombinate_cells", "mutate_cells",
             "diffuse_molecules", "degrade_molecules", "increment_cell_lifetimes"):
    f = getattr(ms.World, name)

    def wrap(self, *a, _f=f, _n=name, **k):
        t0 = time.perf_counter()
        r = _f(self, *a, **k)
        ops[_n] += time.perf_counter() - t0
        return r

    setattr(ms.World, name, wrap)
t0 = time.perf_counter()
for _ in range(steps):
    bench.step(w, 50000, 500, atp)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"{steps} steps: {dt / steps * 1e3:.3f} ms/step")
for k in acc:
    print(f"  {k:28s} {acc[k] / steps * 1e6:8.1f} us/step  ({cnt[k] / steps:.1f}/step)")
for k, v in sorted(ops.items(), key=lambda kv: -kv[1]):
    print(f"  op {k:25s} {v / steps * 1e6:8.1f} us/step host (includes waits)")
