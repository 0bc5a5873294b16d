"""Where performance/check.py's update_cells time goes (10k cells x ~1 kbp on the GPU): the
materialisation of world.cell_genomes, the (genome, index) pairs, update_cells' host work and the
device work it queued. Also per-rep times of the list-API mutations part."""
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def genomes(n, s, d=0.1):
    pop = [-int(s * d), s, int(s * d)]
    return [ms.random_genome(s + random.choice(pop)) for _ in range(n)]


def t():
    torch.cuda.synchronize()
    return time.perf_counter()


# garbage-collector pauses (generation 2 collections walk every tracked object of the process)
import gc  # noqa: E402

_gc = {"t0": 0.0, "total": 0.0, "n2": 0}


def _gc_cb(phase, info):
    if phase == "start":
        _gc["t0"] = time.perf_counter()
    else:
        _gc["total"] += time.perf_counter() - _gc["t0"]
        _gc["n2"] += info.get("generation") == 2


gc.callbacks.append(_gc_cb)


for rep in range(6):
    w = ms.World(chemistry=CHEMISTRY, device="cuda")
    w.spawn_cells(genomes=genomes(10_000, 1000))
    t0 = t()
    _gc["total"], _gc["n2"] = 0.0, 0
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
          f"total {1e3 * (t4 - t0):.1f} (gc {1e3 * _gc['total']:.1f} ms, {_gc['n2']} full)", flush=True)

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
