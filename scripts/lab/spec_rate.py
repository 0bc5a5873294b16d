"""How often does the reference's global early exit of the equilibrium damping (kinetics.py:846)
cut a part short? Runs bench steps and reads the integrator's per-part iteration flags after every
enzymatic_activity: a step counts as "full" when every part ran all 4 iterations (some cell still
had an impactful correction at each of them).

usage: python scripts/lab/spec_rate.py [map_size] [cells] [steps] [chemistry]"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
chem = bench._chemistry(sys.argv[4] if len(sys.argv) > 4 else "wood_ljungdahl")
atp = chem.molname_2_idx.get("ATP", 0)
ms.set_seed(0)
torch.manual_seed(0)
world = ms.World(chemistry=chem, map_size=S, device="cuda:0", seed=0)
world.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
hist = collections.Counter()
orig = world.enzymatic_activity


def act():
    orig()
    m = hip_ops._scratch(world.kinetics).bufs["masks"][:12].view(3, 4).tolist()
    hist[tuple(sum(1 << i for i, v in enumerate(r) if v) for r in m)] += 1


world.enzymatic_activity = act
for _ in range(steps):
    bench.step(world, N, 500, atp)
torch.cuda.synchronize()
full = hist.get((15, 15, 15), 0)
print(f"{S}^2 / {N} cells: {full}/{steps} steps with all parts at 4 iterations; masks {dict(hist)}")
