"""Which Python calls issue device copies in a flagship step: cProfile over a few steps, then the
callers of the tensor methods / functions that copy (copy_, clone, contiguous, to, cat, ...).

    python scripts/lab/copy_probe.py [map_size] [cells] [warmup] [steps]
"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
    warm = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 10
    ms.set_seed(0)
    torch.manual_seed(0)
    bench._prime_rare_paths(CHEMISTRY, "cuda:0", torch.float32, 500)
    w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda:0", seed=0)
    w.spawn_cells(bench.random_genomes(N, 500, "cuda:0"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(warm):
        bench.step(w, N, 500, atp)
    w.synchronize()
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(steps):
        bench.step(w, N, 500, atp)
    prof.disable()
    w.synchronize()
    buf = io.StringIO()
    st = pstats.Stats(prof, stream=buf)
    pat = r"copy_|clone|contiguous|'to' of|\bcat\b|index_select|index_copy|index_put|masked|nonzero|zero_|fill_|full|zeros|empty"
    st.print_callers(pat)
    print(buf.getvalue())


if __name__ == "__main__":
    main()
