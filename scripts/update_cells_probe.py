"""Where performance/check.py's update_cells time goes (10k cells x ~1 kbp on the GPU): the
materialisation of world.cell_genomes, the (genome, index) pairs, update_cells' host work and the
device work it queued. Also per-rep times of the list-API mutations part."""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def genomes(n, s, d=0.1):
    pop = [-int(s * d), s, int(s * d)]
    return [ms.random_genome(s + random.choice(pop)) for _ in range(n)]


def t():
    torch.cuda.synchronize()
    return time.perf_counter()


for rep in range(6):
    w = ms.World(chemistry=CHEMISTRY, device="cuda")
    w.spawn_cells(genomes=genomes(10_000, 1000))
    t0 = t()
    gs = list(w.cell_genomes)
    t1 = t()
    pairs = [(g, i) for i, g in enumerate(gs)]
    t2 = t()
    w.update_cells(pairs)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    w._reconcile()
    t5 = t()
    print(f"rep {rep}: materialise {1e3 * (t1 - t0):.1f} ms, pairs {1e3 * (t2 - t1):.1f}, update host "
          f"{1e3 * (t3 - t2):.1f}, device {1e3 * (t4 - t3):.1f}, reconcile {1e3 * (t5 - t4):.1f}; "
          f"total {1e3 * (t4 - t0):.1f}", flush=True)

if os.environ.get("PROBE_PROFILE") == "1":
    import cProfile
    import pstats

    w = ms.World(chemistry=CHEMISTRY, device="cuda")
    w.spawn_cells(genomes=genomes(10_000, 1000))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    w.update_cells([(g, i) for i, g in enumerate(w.cell_genomes)])
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumtime").print_stats(30)

w = ms.World(chemistry=CHEMISTRY, device="cuda")
gen = genomes(10_000, 1000)
w.spawn_cells(genomes=gen)
gen = list(w.cell_genomes)
for rep in range(6):
    t0 = t()
    ms.point_mutations(seqs=gen)
    t1 = t()
    pairs = w.get_neighbors(cell_idxs=list(range(w.n_cells)))
    t2 = t()
    ms.recombinations(seq_pairs=[(gen[a], gen[b]) for a, b in pairs])
    t3 = t()
    print(f"mutations rep {rep}: point {1e3 * (t1 - t0):.1f} ms, neighbours {1e3 * (t2 - t1):.1f}, "
          f"recombinations {1e3 * (t3 - t2):.1f} ({len(pairs)} pairs); total {1e3 * (t3 - t0):.1f}", flush=True)
