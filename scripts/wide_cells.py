"""Which cells leave the integrator's 32-lane register path on the flagship run (4096^2, 50k)?
After each bench step: the first-level wide count (cells the 32-lane / 16-non-zero launch lists),
the second-level count (cells the 64-lane / 32-non-zero launch lists for the LDS path), and for the
listed cells their active-protein count, most non-zeros of an active protein and largest exponent.

    python scripts/wide_cells.py [steps]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    cells = 50_000
    w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for i in range(steps):
        bench.step(w, cells, 500, atp)
        w.enzymatic_activity()
        torch.cuda.synchronize()
        c = w.n_cells
        kin = w.kinetics
        lists = hip_ops._scratch(kin).bufs["bin_lists"]
        n1, n2 = int(lists[2 * c + 1]), int(lists[2 * c])
        rec = {"step": i, "cells": c, "P": int(kin.N.size(1)), "wide": n1, "wide2": n2}
        if n1:
            idx = lists[c : c + n1].long()
            act = kin.Vmax[idx] > 0
            act |= torch.isnan(kin.Vmax[idx])
            N = kin.N[idx]
            nz = ((N != 0).sum(2) * act).amax(1)
            ex = torch.maximum(kin.Nf[idx].abs().amax((1, 2)), kin.Nb[idx].abs().amax((1, 2)))
            rec["na"] = act.sum(1).tolist()[:20]
            rec["nz_max"] = nz.tolist()[:20]
            rec["exp_max"] = ex.tolist()[:20]
            rec["nan_vmax"] = int(torch.isnan(kin.Vmax[idx]).any(1).sum())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
