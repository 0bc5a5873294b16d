"""Integrator timing breakdown on the flagship state (4096^2 map, 50k cells after a few steps):
per-call times of enzymatic_activity and of explicit-X integrations with 1 or 3 parts and 0 or 4
damping iterations, plus the active-protein distribution that sizes the LDS slots."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import kinetics_ops  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / iters * 1e3, 1)


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    cells = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
    w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(5):
        bench.step(w, cells, 500, atp)
    kin = w.kinetics
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    out = {"cells": w.n_cells, "P": int(kin.N.size(1)), "s": int(kin.N.size(2))}
    na = (kin.Vmax > 0).sum(1)
    out["active_mean"] = round(float(na.float().mean()), 2)
    out["active_hist"] = {str(k): int((na == k).sum()) for k in range(0, int(na.max()) + 1)}
    nz = ((kin.N != 0).sum(2) * (kin.Vmax > 0)).amax(1)  # most non-zero signals of an active protein
    out["wide_cells_nz16"] = int((nz > 16).sum())
    out["wide_cells_nz32"] = int((nz > 32).sum())
    out["us_enzymatic_activity"] = timed(w.enzymatic_activity)
    from magicsoup_amd.ops import native

    for rep_i in range(3):  # A/B of the launch modes on the same state (alternating)
        # speculative all-parts launch; per-part register launches; + unfused wide list; + sort
        for mode in (0, 256, 128, 64):
            native.hip().set_integrate_mode(mode)
            Xk = X.clone()
            out[f"us_mode{mode}_r{rep_i}"] = timed(lambda: kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), 4))
    res = {}
    for mode in (0, 8, 9, 10, 11, 12, 16, 32, 64, 128, 256):  # every mode computes the same state, bit for bit
        native.hip().set_integrate_mode(mode)
        Xk = X.clone()
        kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), 4)
        res[mode] = Xk
    out["modes_equal"] = {m: bool(torch.equal(res[0], v)) for m, v in res.items()}
    out["max_abs_diff_legacy"] = float((res[0] - res[8]).abs().max())
    out["us_ea_sorted"] = (native.hip().set_integrate_mode(16), timed(w.enzymatic_activity))[1]
    out["us_ea_per_part"] = (native.hip().set_integrate_mode(128), timed(w.enzymatic_activity))[1]
    out["us_ea_spec_snap_writeback"] = (native.hip().set_integrate_mode(256), timed(w.enzymatic_activity))[1]
    native.hip().set_integrate_mode(0)
    out["us_ea_spec_direct"] = timed(w.enzymatic_activity)
    out["us_ea_spec_snap_writeback_2"] = (native.hip().set_integrate_mode(256), timed(w.enzymatic_activity))[1]
    native.hip().set_integrate_mode(0)
    out["us_ea_fast"] = timed(w.enzymatic_activity)
    native.hip().set_integrate_mode(0)
    for trims in ((0.7,), (0.7, 0.2, 0.1)):
        for it in (0, 4):
            Xk = X.clone()
            out[f"us_parts{len(trims)}_iters{it}"] = timed(lambda: kinetics_ops.integrate(kin, Xk, trims, it))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
