"""Call order of the World ops and the internal synchronisation points of a few flagship steps
(nesting shown by indentation): where the host waits for the device, and inside which op.

    python scripts/lab/call_order.py [map_size] [cells] [warmup] [steps]
"""
import functools
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.models import world as world_mod  # noqa: E402
from magicsoup_amd.ops import genome_pipeline, hip_ops, streams  # noqa: E402

depth = [0]
on = [False]
t0 = [0.0]


def trace(owner, name):
    f = getattr(owner, name)

    @functools.wraps(f)
    def w(*a, **k):
        if not on[0]:
            return f(*a, **k)
        t = time.perf_counter()
        print(f"{(t - t0[0]) * 1e6:9.1f} {'  ' * depth[0]}> {owner.__name__}.{name}", flush=True)
        depth[0] += 1
        ret = [None]
        try:
            ret[0] = f(*a, **k)
            return ret[0]
        finally:
            depth[0] -= 1
            e = time.perf_counter()
            print(f"{(e - t0[0]) * 1e6:9.1f} {'  ' * depth[0]}< {owner.__name__}.{name} ({(e - t) * 1e6:.1f} us)"
                  + (f" -> {ret[0]!r}" if name == "_chain_bound" else ""), flush=True)

    setattr(owner, name, w)


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    W = world_mod.World
    for name in ("enzymatic_activity", "kill_divide_where", "diffuse_molecules", "degrade_molecules",
                 "increment_cell_lifetimes", "recombinate_cells", "mutate_cells", "_resolve_count",
                 "_flush_deferred", "_reconcile", "_join_side", "_evolve", "_chain_bound"):
        trace(W, name)
    for name in ("reconcile", "_resolve", "evolve"):
        trace(genome_pipeline, name)
    trace(streams.NEvent, "synchronize")
    trace(hip_ops, "guarded_sync")
    trace(hip_ops, "_launch_integrate")
    ms.set_seed(0)
    torch.manual_seed(0)
    bench._prime_rare_paths(CHEMISTRY, "cuda:0", torch.float32, 500)
    if os.environ.get("MS_VIRTUAL_STRIPS") == "1":  # a one-rank strip world (host_split.py)
        import torch.distributed as dist

        from magicsoup_amd.parallel import DistributedWorld, dist_world

        for name in ("enzymatic_activity", "_resolve_count", "_divide_phase_b", "_divide_mask_native",
                     "kill_divide_where", "_evolve", "diffuse_molecules"):
            if name in DistributedWorld.__dict__:
                trace(DistributedWorld, name)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29548")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        w = DistributedWorld(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0, strips=True)
    else:
        w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda:0", seed=0)
    w.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(warm):
        bench.step(w, N, 500, atp)
    w.synchronize()
    for s in range(steps):
        print(f"---- step {s}", flush=True)
        on[0] = True
        t0[0] = time.perf_counter()
        bench.step(w, N, 500, atp)
        on[0] = False
    w.synchronize()
    print("declined device-count chain issues:", genome_pipeline.BOUND_DECLINED, flush=True)


if __name__ == "__main__":
    main()
