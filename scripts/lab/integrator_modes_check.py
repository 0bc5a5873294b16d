"""Which integrator launch modes agree bit for bit on one state, and which cells differ (with their
active-protein counts): a diagnostic for tests/test_gpu_kernels.py
test_register_integrator_matches_lds_integrator_bit_for_bit.

    python scripts/lab/integrator_modes_check.py [genome_size] [cells]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import kinetics_ops, native  # noqa: E402
from tests.conftest import gen_genomes  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    ms.set_seed(2)
    torch.manual_seed(2)
    w = ms.World(chemistry=CHEMISTRY, map_size=64, device="cuda", seed=2)
    w.spawn_cells(gen_genomes(n, size))
    kin = w.kinetics
    na = (kin.Vmax > 0).sum(1)
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    out, masks = {}, {}
    for mode in (8, 0, 32, 64, 128, 256):
        native.hip().set_integrate_mode(mode)
        Xk = X.clone()
        masks[mode] = kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), 4)
        out[mode] = Xk
    native.hip().set_integrate_mode(0)
    for n_iters in (0,):
        for mode in (8, 0, 128):
            native.hip().set_integrate_mode(mode)
            Xk = X.clone()
            kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), n_iters)
            out[f"{mode}_it{n_iters}"] = Xk
    native.hip().set_integrate_mode(0)
    rep = {"cells": n, "genome": size, "na_max": int(na.max()), "na_gt32": int((na > 32).sum()),
           "na_gt256": int((na > 256).sum()), "masks": {str(k): v for k, v in masks.items()}}
    for key, v in out.items():
        ref = out[8] if not str(key).endswith("_it0") else out["8_it0"]
        bad = (v != ref).any(1).nonzero().flatten().cpu()
        rep[str(key)] = {"n_diff": int(bad.numel()), "na_of_diff": na[bad.to(na.device)][:12].tolist(),
                         "max_abs": float((v - ref).abs().max())}
    print(json.dumps(rep))


if __name__ == "__main__":
    main()


def host_vs_gpu():
    """tests/test_gpu_kernels.py test_enzymatic_activity_matches_host, with the differing cells."""
    import copy

    from tests.test_gpu_kernels import _copy_world_cpu_to_gpu, _world

    wc = _world("cpu", n=300)
    wg = _copy_world_cpu_to_gpu(wc)
    na = (wc.kinetics.Vmax > 0).sum(1)
    for mode in (0, 128, 8):
        native.hip().set_integrate_mode(mode)
        a, b = copy.deepcopy(wc), copy.deepcopy(wg)
        a.enzymatic_activity()
        b.enzymatic_activity()
        ok = torch.isclose(b.cell_molecules.cpu(), a.cell_molecules, rtol=1e-4, atol=1e-4).all(1)
        bad = (~ok).nonzero().flatten()
        print(json.dumps({"mode": mode, "n_bad": int(bad.numel()), "na_bad": na[bad][:10].tolist(),
                          "max_abs": float((b.cell_molecules.cpu() - a.cell_molecules).abs().max())}))
    native.hip().set_integrate_mode(0)


if __name__ == "__main__" and len(sys.argv) > 3:
    host_vs_gpu()
