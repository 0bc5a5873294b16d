"""A/B of the integrator's rescue launch (one launch behind the speculative fused kernel) against
the separate launches, on the flagship state: median enzymatic_activity time (with the world's
state restored between calls) per mode, alternating.

    python scripts/lab/rescue_ab.py [steps_before]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import native  # noqa: E402
from scripts.lab.evolved_probe import timed_activity  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    ms.set_seed(0)
    w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(50_000, 500, "cuda"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(steps):
        bench.step(w, 50_000, 500, atp)
    w.synchronize()
    out = {"cells": w.n_cells}
    for rep in range(3):
        for mode in (1, 0):
            native.hip().set_rescue_mode(mode)
            out.setdefault(f"rescue{mode}", []).append(timed_activity(w, iters=9))
    native.hip().set_rescue_mode(1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
