"""Device translation time of long genomes (the global-slot pass, a workgroup per genome):
hip_ops.translate (count pass, stats, write pass) over a few giant random genomes, median of 20 calls.

usage: python scripts/lab/tlong_bench.py"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.getcwd())  # (the checkout it runs from: an A/B worktree imports its own build)
import torch  # noqa: E402

import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.models.strings import PoolArena, pack_strings  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402

genetics = ms.Genetics()
ms.set_seed(3)
for label, sizes in (("1x200k", [200_000]), ("4x100k", [100_000] * 4), ("32x20k", [20_000] * 32),
                     ("256x4k", [4_000] * 256)):
    arr, lens = pack_strings([ms.random_genome(n) for n in sizes])
    pool = PoolArena("cuda")
    pool.append_packed(torch.from_numpy(arr), torch.from_numpy(lens))
    rows = torch.arange(len(sizes), device="cuda")
    for _ in range(3):
        hip_ops.translate(genetics, pool, rows)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        hip_ops.translate(genetics, pool, rows)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    print({"case": label, "ms_median": round(statistics.median(ts), 3), "ms_min": round(min(ts), 3)}, flush=True)
