"""Phase cycles of the register integrator (a -DMS_INT_PROF build of the module, scripts/lab/
build_variant.py): integrate the bench population on an explicit X a few times and print the cycles of
each phase of the launch's first cell per launch (clock64 deltas, parts summed).

usage: MS_VARIANT_FLAGS=-DMS_INT_PROF python scripts/lab/build_variant.py ab/int_prof.so magicsoup_amd/csrc/hip/kinetics.hip
       python scripts/lab/int_prof.py ab/int_prof.so [size] [cells]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.ops import hip_ops, kinetics_ops, native  # noqa: E402
from scripts.lab.ab_so import load  # noqa: E402

NAMES = ["x0", "active", "loads", "unpack", "velocity", "consumption", "factor", "advance0", "damping", "writeback"]
path = sys.argv[1]
size = int(sys.argv[2]) if len(sys.argv) > 2 else 64
cells = int(sys.argv[3]) if len(sys.argv) > 3 else 200
mod = load(path, "prof")
chem = bench._chemistry("wl")
w = ms.World(chemistry=chem, map_size=size, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
for _ in range(5):
    bench.step(w, cells, 500, chem.molname_2_idx["ATP"])
w.synchronize()
kin = w.kinetics
pos = w.cell_positions.long()
X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
kin._packed_params()
native._mods["_hip"] = hip_ops._MOD = mod
mod.int_prof_read(True)
for _ in range(20):
    Xk = X.clone()
    kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), 4)
v = mod.int_prof_read(True)
n = max(1, v[63])
out = {"cells": w.n_cells, "launches": n, **{NAMES[i]: round(v[i] / n) for i in range(10)}}
out["total"] = sum(out[k] for k in NAMES)
print(json.dumps(out))
