"""Active-protein histogram of the flagship bench world after some steps (integrator binning)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402

chem = bench._chemistry("wl")
atp = chem.molname_2_idx["ATP"]
ms.set_seed(1)
torch.manual_seed(1)
w = ms.World(chemistry=chem, map_size=4096, device="cuda", seed=1)
w.spawn_cells(bench.random_genomes(50000, 500, "cuda"))
for i in range(40):
    bench.step(w, 50000, 500, atp)
    if i % 10 == 9:
        na = (w.kinetics.Vmax > 0).sum(1)
        h = torch.bincount(na.cpu(), minlength=1)
        print(f"step {i+1}: P={w.kinetics.Vmax.size(1)} n={w.n_cells} >12: {int((na > 12).sum())} >16: {int((na > 16).sum())} "
              f"max={int(na.max())} mean={float(na.float().mean()):.1f} hist={h.tolist()[:40]}", flush=True)
