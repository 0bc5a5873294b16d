"""Kinetics parameters of the same genomes derived on the host (CPU world moved to the GPU) and by the
device pipeline (GPU world spawning them): which parameters differ, and by how many ulps.

usage: python scripts/lab/param_paths.py [cells]"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import genome_pipeline  # noqa: E402
from tests.conftest import gen_genomes  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 700
ms.set_seed(4)
torch.manual_seed(4)
g = ms.World(chemistry=CHEMISTRY, map_size=256 if n > 3000 else 64, seed=4, device="cpu")
g.spawn_cells(gen_genomes(n, 300))
a = copy.deepcopy(g).to("cuda")  # host-derived parameters, moved
b = copy.deepcopy(g).to("cuda")
rows = torch.arange(b.n_cells, device="cuda")
if not genome_pipeline.rebuild_rows(b, rows):  # device translation + build of every cell
    b._update_params_rows(rows)
b.synchronize()
ka, kb = a.kinetics, b.kinetics
for name in ("N", "Nf", "Nb", "A", "Kmf", "Kmb", "Kmr", "Vmax", "Ke"):
    x = getattr(ka, name).cpu()
    y = getattr(kb, name).cpu()
    P = min(x.size(1), y.size(1))
    x, y = x[:, :P], y[:, :P]
    d = x != y
    cells = int(d.reshape(d.size(0), -1).any(dim=1).sum())
    rel = 0.0
    if x.is_floating_point() and d.any():
        rel = float(((x - y).abs() / x.abs().clamp(min=1e-30))[d].max())
    print(f"{name:5s} cells differing {cells:5d} entries {int(d.sum()):6d} max rel {rel:.3g}")
