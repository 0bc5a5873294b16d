"""Per-op launch counts, device time and host time of the flagship step (torch.profiler on ROCm).

usage: python scripts/op_launches.py [map_size] [cells] [steps]"""
import os
import sys
import time
from collections import defaultdict

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(5):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()


class T:
    def __init__(self):
        self.host = defaultdict(float)
        self.cur = None

    def phase(self, name):
        t = self

        class C:
            def __enter__(self):
                torch.cuda.synchronize()
                self.t0 = time.perf_counter()
                self.r = torch.profiler.record_function("PH_" + name)
                self.r.__enter__()

            def __exit__(self, *a):
                self.r.__exit__(*a)
                t.host[name] += time.perf_counter() - self.t0  # host time to issue (no sync)
                torch.cuda.synchronize()

        return C()


timer = T()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(steps):
        bench.step(w, N, 500, atp, timer=timer)
    torch.cuda.synchronize()

# attribute device kernels to phases through their launching CPU op's time range
evs = prof.events()
ranges = [(e.time_range.start, e.time_range.end, e.name[3:]) for e in evs if e.name.startswith("PH_")]
kern = defaultdict(int)
ktime = defaultdict(float)
for e in evs:
    if e.device_type == torch.autograd.DeviceType.CUDA:
        # kineto links kernels to the launching runtime call; fall back to the kernel's own start
        t = e.time_range.start
        for a, b, nm in ranges:
            if a <= t <= b + 2000:
                kern[nm] += 1
                ktime[nm] += e.time_range.elapsed_us()
                break
print(f"{'phase':14s} {'host_ms':>8s} {'launch/step':>11s} {'dev_us/step':>11s}")
for nm in timer.host:
    print(f"{nm:14s} {timer.host[nm] / steps * 1e3:8.3f} {kern[nm] / steps:11.1f} {ktime[nm] / steps:11.1f}")
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=40))
