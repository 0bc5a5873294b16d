"""Speculative single-process integration (fused launch + rescue) against the decomposed-world
protocol (speculative launch, flag hook, per-part launches) on the same world state, in one process:
which cells differ, and their proteome shapes.

usage: python scripts/lab/int_paths.py [cells] [map_size] [seed]"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402
from tests.conftest import gen_genomes  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 700
S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 4
ms.set_seed(seed)
torch.manual_seed(seed)
g = ms.World(chemistry=CHEMISTRY, map_size=S, seed=seed, device="cpu")
g.spawn_cells(gen_genomes(n, 300))
a = copy.deepcopy(g).to("cuda")
b = copy.deepcopy(g).to("cuda")
a.enzymatic_activity()
kin = b.kinetics
p = kin._packed_params()
hip_ops._ensure_world_layout(b)
hip_ops._launch_integrate(kin, p, b.n_cells, world=b, flags_hook=lambda t: None, slot=kin._slot_tensor())
torch.cuda.synchronize()
ca, cb = a.cell_molecules.cpu(), b.cell_molecules.cpu()
bad = torch.nonzero((ca != cb).any(dim=1)).flatten().tolist()
print("cells", n, "differing", len(bad), "map equal", torch.equal(a.molecule_map.cpu(), b.molecule_map.cpu()))
N = kin.N.cpu()
V = kin.Vmax.cpu()
for i in bad[:10]:
    act = int((V[i] != 0).sum())
    nz = (N[i] != 0).sum(dim=1)
    print(f"  cell {i}: proteins {int(kin._nprot()[i]) if hasattr(kin, '_nprot') else N.size(1)} active {act} "
          f"max non-zeros {int(nz.max())} max |d| {float((ca[i] - cb[i]).abs().max()):.3g}")
