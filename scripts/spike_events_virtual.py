"""Slow steps of a one-rank strip world (MS_VIRTUAL_STRIPS-style: the multi-GPU protocol against
itself over RCCL) and the methods that ran more often than usual in them: every method of World,
DistributedWorld, Kinetics, StringArena and the op modules is counted per step.

usage: python scripts/spike_events_virtual.py [map_size] [cells] [steps] [warmup]"""
import collections
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29577")
torch.cuda.set_device(0)
torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.parallel import DistributedWorld  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1448
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6250
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 5
counts = collections.Counter()


def wrap(f, key):
    def w(*a, **k):
        counts[key] += 1
        return f(*a, **k)
    return w


import importlib  # noqa: E402

for modname, clsname in [("magicsoup_amd.models.world", "World"), ("magicsoup_amd.parallel.dist_world", "DistributedWorld"),
                         ("magicsoup_amd.models.kinetics", "Kinetics"), ("magicsoup_amd.models.strings", "StringArena"),
                         ("magicsoup_amd.ops.hip_ops", None), ("magicsoup_amd.ops.genome_pipeline", None)]:
    mod = importlib.import_module(modname)
    owner = getattr(mod, clsname) if clsname else mod
    for name, val in list(vars(owner).items()):
        if (callable(val) and not isinstance(val, (type, staticmethod, classmethod)) and not name.startswith("__")
                and getattr(val, "__module__", "") == modname):
            setattr(owner, name, wrap(val, f"{clsname or modname.split('.')[-1]}.{name}"))

atp = CHEMISTRY.molname_2_idx["ATP"]
w = DistributedWorld(chemistry=CHEMISTRY, map_size=S, device="cuda:0", seed=0, strips=True)
bench._prime_rare_paths(CHEMISTRY, "cuda:0", torch.float32, 500)
w.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
for _ in range(warm):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
recs = []
for _ in range(steps):
    counts.clear()
    t0 = time.perf_counter()
    bench.step(w, N, 500, atp)
    torch.cuda.synchronize()
    recs.append(((time.perf_counter() - t0) * 1e3, dict(counts)))
med = statistics.median(t for t, _ in recs)
typical = collections.defaultdict(list)
for _, c in recs:
    for k in set().union(*(r[1] for r in recs)):
        typical[k].append(c.get(k, 0))
base = {k: statistics.median(v) for k, v in typical.items()}
print(f"{S}^2 / {N} virtual strips: {steps} steps (synchronised), median {med:.3f} ms")
for i, (t, c) in enumerate(recs):
    if t > 2 * med:
        extra = {k: v for k, v in c.items() if v > base.get(k, 0)}
        print(f"  step {i:3d} {t:8.3f} ms  more than usual: {extra}")
w.close()
torch.distributed.destroy_process_group()
