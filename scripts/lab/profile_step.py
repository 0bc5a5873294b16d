"""Host-side profile of the flagship step: per-op host time (perf_counter around each World op, no
synchronisation added) and a cProfile of the same steps, top functions by self time.

usage: python scripts/lab/profile_step.py [map_size] [cells] [steps]
MS_VIRTUAL_STRIPS=1: profile a one-rank DistributedWorld running the strip protocol (RCCL to itself)."""
import collections
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

map_size = int(sys.argv[1]) if len(sys.argv) > 1 else 256
cells = int(sys.argv[2]) if len(sys.argv) > 2 else 40000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = "cuda" if torch.cuda.is_available() else "cpu"
if os.environ.get("MS_VIRTUAL_STRIPS") == "1":
    import torch.distributed as dist

    from magicsoup_amd.parallel import DistributedWorld

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    if dev == "cuda":
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=0, world_size=1)
    w = DistributedWorld(chemistry=CHEMISTRY, map_size=map_size, device=dev, seed=0, strips=True)
else:
    w = ms.World(chemistry=CHEMISTRY, map_size=map_size, device=dev, seed=0)
w.spawn_cells(bench.random_genomes(cells, 500, dev))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(5):
    bench.step(w, cells, 500, atp)
if dev == "cuda":
    torch.cuda.synchronize()

# per-op host time (includes the op's own synchronisations, e.g. kill's count read-back)
acc = collections.defaultdict(float)
names = ("spawn_cells", "enzymatic_activity", "kill_cells", "divide_cells_t", "recombinate_cells", "mutate_cells",
         "degrade_molecules", "diffuse_molecules", "increment_cell_lifetimes")
cls = type(w)
orig = {}
for nm in names:
    f = getattr(cls, nm)
    orig[nm] = f

    def wrap(self, *a, _f=f, _n=nm, **k):
        t0 = time.perf_counter()
        try:
            return _f(self, *a, **k)
        finally:
            acc[_n] += time.perf_counter() - t0

    setattr(cls, nm, wrap)
t0 = time.perf_counter()
for _ in range(steps):
    bench.step(w, cells, 500, atp)
t_host = time.perf_counter() - t0
if dev == "cuda":
    torch.cuda.synchronize()
t_all = time.perf_counter() - t0
for nm, f in orig.items():
    setattr(cls, nm, f)
print(f"{steps} steps: {t_all / steps * 1e3:.3f} ms/step wall, host loop {t_host / steps * 1e3:.3f} ms/step")
tot = 0.0
for nm in names:
    tot += acc[nm]
    print(f"  {nm:26s} {acc[nm] / steps * 1e3:8.3f} ms/step")
print(f"  {'(bench code between ops)':26s} {(t_host - tot) / steps * 1e3:8.3f} ms/step")

pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    bench.step(w, cells, 500, atp)
if dev == "cuda":
    torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(50)
st.sort_stats("cumulative").print_stats(60)
