"""Host time of World ops on the flagship world with the device otherwise idle: a call that takes
about as long as its kernels run means a launch inside it waited for the device."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402

w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(50000, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(5):
    bench.step(w, 50000, 500, atp)
x = torch.zeros(16, device="cuda")
for name, fn in [("diffuse", w.diffuse_molecules), ("activity", w.enzymatic_activity),
                 ("degrade", w.degrade_molecules)]:
    res = []
    for _ in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        x.add_(1.0)
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        res.append((round((t1 - t0) * 1e6), round((t2 - t1) * 1e6), round((t3 - t0) * 1e6)))
    print(name, "host call / next launch / wall (us):", res)
# the stencil launcher alone
d = w.__dict__
res = []
for _ in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hip_ops.diffuse(w)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    res.append(round((t1 - t0) * 1e6))
print("hip_ops.diffuse host:", res)
