"""Synchronous-path translation of 10k x ~1 kbp genomes (performance/check.py update_cells): the
token tensor's shape and the time of each pass, repeated, to find what makes some write passes
70x slower than others (profiles/r4/tcheck)."""
import os
import random
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402


def genomes(n, s, d=0.1):
    pop = [-int(s * d), s, int(s * d)]
    return [ms.random_genome(s + random.choice(pop)) for _ in range(n)]


for rep in range(6):
    w = ms.World(chemistry=CHEMISTRY, device="cuda")
    w.spawn_cells(genomes=genomes(10_000, 1000))
    w._reconcile()
    torch.cuda.synchronize()
    rows = torch.arange(w.n_cells, device="cuda")
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    tokens, nprot = hip_ops.translate(w.genetics, w._genomes, rows)
    b.record()
    torch.cuda.synchronize()
    t_first = a.elapsed_time(b)
    a.record()
    tokens2, _ = hip_ops.translate(w.genetics, w._genomes, rows)  # the same genomes again
    b.record()
    torch.cuda.synchronize()
    same = torch.equal(tokens, tokens2)
    lens = w._genomes.lens[: w.n_cells]
    print(f"rep {rep}: tokens {tuple(tokens.shape)} = {tokens.numel() * 4 / 2**20:.0f} MiB, translate "
          f"{t_first:.2f} ms, again {a.elapsed_time(b):.2f} ms (same {same}), genomes > 1024 nt: "
          f"{int((lens > 1024).sum())}, width {w._genomes.width}", flush=True)
    del tokens, nprot, w
