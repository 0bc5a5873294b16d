"""cProfile of pipelined bench steps (host-side cost by function, self time first).

usage: python scripts/step_cprofile.py [map_size] [cells] [steps] [sort]
MS_VIRTUAL_STRIPS=1: a one-rank DistributedWorld running the strip protocol (RCCL to itself)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1448
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6250
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
sort = sys.argv[4] if len(sys.argv) > 4 else "tottime"
virtual = os.environ.get("MS_VIRTUAL_STRIPS") == "1"
if virtual:
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from magicsoup_amd.parallel import DistributedWorld

    w = DistributedWorld(chemistry=CHEMISTRY, map_size=S, device="cuda:0", seed=0, strips=True)
else:
    w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda:0", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(30):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
pr = cProfile.Profile()
import time  # noqa: E402

t0 = time.perf_counter()
pr.enable()
for _ in range(steps):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
pr.disable()
dt = time.perf_counter() - t0
print(f"{S}^2 / {N} {'virtual' if virtual else 'plain'}: {dt / steps * 1e6:.0f} us per step under cProfile")
st = pstats.Stats(pr)
st.sort_stats(sort).print_stats(int(os.environ.get("MS_PROF_LINES", "45")))
if virtual:
    w.close()
