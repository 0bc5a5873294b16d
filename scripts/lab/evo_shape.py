"""Why evolved chains ask for host rebuilds: after some evolving flagship steps, the proteome shape
against the device pipeline's speculative token layout (genome_pipeline.D_CAP domains per protein,
the kinetics' protein bound P) -- cells past it are the ones the chain lists for the host rebuild
(gp.hip gp_check_assign_kernel) -- and how often the chains' flags fired.

usage: python scripts/lab/evo_shape.py [steps]"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import genome_pipeline as gp  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
w = ms.World(chemistry=CHEMISTRY, map_size=4096, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(50_000, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
flags = collections.Counter()
listed = []
orig = gp._rebuild_set


def spy(pd):
    f = int(pd.host[1])
    flags[f] += 1
    r = orig(pd)
    if f & gp._F_PARTIAL and r is not None:
        listed.append(int(r.numel()))
    return r


gp._rebuild_set = spy
for i in range(steps):
    bench.step(w, 50_000, 500, atp)
    if i in (steps // 2, steps - 1):
        w.synchronize()
        print({"step": i, "flags": dict(flags), "listed_mean": sum(listed) / max(len(listed), 1),
               "listed_max": max(listed, default=0)}, flush=True)
        flags.clear()
        listed.clear()
w.synchronize()
from magicsoup_amd.ops import hip_ops  # noqa: E402

rows = torch.arange(w.n_cells, device="cuda")
arena = w._genomes
n = w.n_cells
tok, nprot = hip_ops.translate(w.genetics, arena, rows)
doms = (tok[..., 0] != 0).sum(-1)  # (n, P) domains per protein
lens = arena.lens[:n]
print({"cells": n, "P": w.kinetics._P(), "token_D": tok.size(2), "max_nprot": int(nprot.max()),
       "cells_nprot_gt_P": int((nprot > w.kinetics._P()).sum()),
       "max_domains": int(doms.max()), "cells_dom_gt_DCAP": int((doms > gp.D_CAP).any(1).sum()),
       "max_genome": int(lens.max()), "genomes_gt_2048": int((lens > 2048).sum()),
       "genomes_gt_10k": int((lens > 10000).sum())}, flush=True)
big = (doms > gp.D_CAP).any(1)
if big.any():
    print({"len_of_dom_overflow_cells": lens[big][:20].tolist()}, flush=True)
