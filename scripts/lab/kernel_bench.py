"""Isolated hot-kernel workload for counter collection: a 50k-cell world on a 4096^2 map, then a
few enzymatic_activity / diffuse / kill+divide rounds (each op synchronised)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    cells = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(3):  # reach a steady population / protein width
        bench.step(w, cells, 500, atp)
    torch.cuda.synchronize()
    for name, fn in (("enzymatic_activity", w.enzymatic_activity), ("diffuse", w.diffuse_molecules)):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        print(f"{name}: {(time.perf_counter() - t0) / iters * 1e3:.3f} ms", flush=True)
    print(f"cells={w.n_cells} P={w.kinetics.N.size(1)} s={w.kinetics.N.size(2)}")


if __name__ == "__main__":
    main()
