"""Inclusive host time per call of selected internal functions inside pipelined bench steps (no
synchronisation added): where the host spends a step.

usage: python scripts/lab/host_breakdown.py [map_size] [cells] [steps]
MS_VIRTUAL_STRIPS=1: a one-rank DistributedWorld running the strip protocol (RCCL to itself)."""
import collections
import importlib
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
TARGETS = [
    ("magicsoup_amd.models.world", "World", "_flush_deferred"),
    ("magicsoup_amd.models.world", "World", "_reconcile"),
    ("magicsoup_amd.models.world", "World", "_divide_mask_gpu"),
    ("magicsoup_amd.models.world", "World", "kill_cells"),
    ("magicsoup_amd.models.world", "World", "enzymatic_activity"),
    ("magicsoup_amd.models.world", "World", "spawn_cells"),
    ("magicsoup_amd.ops.genome_pipeline", None, "point_mutations"),
    ("magicsoup_amd.ops.genome_pipeline", None, "recombinate_all"),
    ("magicsoup_amd.ops.genome_pipeline", None, "reconcile"),
    ("magicsoup_amd.ops.genome_pipeline", None, "_kin_desc"),
    ("magicsoup_amd.ops.genome_pipeline", None, "_begin"),
    ("magicsoup_amd.ops.genome_pipeline", None, "_record"),
    ("magicsoup_amd.ops.hip_ops", None, "neighbor_slot_keys"),
    ("magicsoup_amd.ops.hip_ops", None, "enzymatic_activity"),
    ("magicsoup_amd.ops.hip_ops", None, "wait_count"),
    ("magicsoup_amd.ops.hip_ops", None, "gather_rows"),
    ("magicsoup_amd.ops.hip_ops", None, "divide_mask_issue"),
    ("magicsoup_amd.ops.hip_ops", None, "diffuse"),
    ("magicsoup_amd.ops.hip_ops", None, "spill_and_free_mask"),
    ("magicsoup_amd.ops.hip_ops", None, "select_async"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "divide_cells_t"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "recombinate_cells"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "_exchange"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "_do_exchange_map_halo"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "_do_allreduce_flags"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "_do_allreduce_totals"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "_append_arrivals"),
    ("magicsoup_amd.parallel.dist_world", "DistributedWorld", "_clone_rows"),
    ("magicsoup_amd.parallel.strip", None, "marks"),
    ("magicsoup_amd.parallel.strip", None, "reserve"),
    ("magicsoup_amd.parallel.strip", None, "split_winners_gpu"),
    ("magicsoup_amd.parallel.strip", None, "pack"),
    ("magicsoup_amd.parallel.strip", None, "clear"),
]
acc = collections.defaultdict(lambda: [0.0, 0])


def wrap(f, key):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            e = acc[key]
            e[0] += time.perf_counter() - t0
            e[1] += 1
    return w


if os.environ.get("MS_VIRTUAL_STRIPS") == "1":
    import torch.distributed as dist

    from magicsoup_amd.parallel import DistributedWorld

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29543")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    w = DistributedWorld(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0, strips=True)
else:
    w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(20):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
for mod, cls, fn in TARGETS:
    m = importlib.import_module(mod)
    owner = getattr(m, cls) if cls else m
    setattr(owner, fn, wrap(getattr(owner, fn), f"{cls + '.' if cls else mod.split('.')[-1] + '.'}{fn}"))
t0 = time.perf_counter()
for _ in range(steps):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps * 1e6
print(f"{S}^2 / {N}: {dt:.0f} us per step; inclusive host us per step (calls per step)")
for key, (t, c) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
    print(f"  {key:40s} {t / steps * 1e6:8.1f}  ({c / steps:.2f})")
