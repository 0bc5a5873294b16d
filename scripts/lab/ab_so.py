"""A/B two builds of the _hip extension on one world state, in one process: the flagship world is
built with the in-tree module, then an integrate (3 parts, 4 iterations) on the same explicit X is
timed alternately with module A and module B, and their results are compared bit for bit.

Each module is timed in every integrate mode of --modes (comma list, default 0); results must be
bit-identical across modules and modes.

usage: python scripts/lab/ab_so.py [--size S] [--cells C] [--chem wl|synthetic:M:R] [--modes 0,128] [--steps K] [--iters I]
                               A.so B.so [C.so ...]"""
import importlib.machinery
import importlib.util
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.ops import kinetics_ops, native  # noqa: E402


def load(path, tag):
    # the in-tree module itself: a second load of the same file would re-run its module init on the
    # same shared object (pybind11 refuses the repeated class registrations)
    if os.path.realpath(path) == os.path.realpath(native.hip().__file__):
        return native.hip()
    name = f"ab_{tag}._hip"
    loader = importlib.machinery.ExtensionFileLoader(name, path)
    spec = importlib.util.spec_from_loader(name, loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


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
    args = sys.argv[1:]
    size, cells, chem_spec, modes, steps, iters = 4096, 50000, "wl", [0], 5, 4
    while args and args[0].startswith("--"):
        flag, val = args[0], args[1]
        args = args[2:]
        if flag == "--size":
            size = int(val)
        elif flag == "--cells":
            cells = int(val)
        elif flag == "--chem":
            chem_spec = val
        elif flag == "--steps":
            steps = int(val)
        elif flag == "--iters":
            iters = int(val)
        else:
            modes = [int(v) for v in val.split(",")]
    mods = {chr(65 + i): load(p, f"v{i}") for i, p in enumerate(args)}
    chem = bench._chemistry(chem_spec)
    atp = chem.molname_2_idx.get("ATP", 0)
    w = ms.World(chemistry=chem, map_size=size, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
    for _ in range(steps):
        bench.step(w, cells, 500, atp)
    w.synchronize()
    kin = w.kinetics
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    kin._packed_params()
    out, res = {"P": int(kin._P()), "cells": w.n_cells}, {}
    from magicsoup_amd.ops import hip_ops

    orig = native._mods.get("_hip")
    try:
        for rep in range(3):
            for tag, mod in mods.items():
                # (hip_ops caches the module it resolved first: swap both handles)
                native._mods["_hip"] = hip_ops._MOD = mod
                for mode in modes:
                    mod.set_integrate_mode(mode)
                    Xk = X.clone()
                    out[f"{tag}_m{mode}_r{rep}"] = timed(lambda: kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), iters))
                    Xk = X.clone()
                    kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), iters)
                    res[f"{tag}_m{mode}"] = Xk
                mod.set_integrate_mode(0)
        first = next(iter(res.values()))
        out["equal"] = {t: bool(torch.equal(first, r)) for t, r in res.items()}
    finally:
        native._mods["_hip"] = hip_ops._MOD = orig
    print(json.dumps(out))


if __name__ == "__main__":
    main()
