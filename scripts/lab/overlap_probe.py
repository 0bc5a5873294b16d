"""How much of the diffusion stencil can hide behind the enzymatic activity: time the flagship
world's activity alone, the stencil alone, and both issued at once on two streams (timing only:
the concurrent run races on the pixels under cells, its results are discarded).
usage: python scripts/lab/overlap_probe.py [size] [cells] [iters]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402
from magicsoup_amd.ops.hip_ops import _m, _mdt, _p, _scratch, geom  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    cells = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=0)
    w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(10):
        bench.step(w, cells, 500, atp)
    w.synchronize()
    torch.cuda.synchronize()
    d = w.__dict__
    hip_ops.apply_pending(w)
    mm = d["_molmap"]
    m = int(mm.size(0))
    R, C, r_lo, r_hi, wrap = geom(w)
    sc = _scratch(w)
    tmp = sc.get("diff_tmp", mm.numel(), mm.dtype, mm.device)
    partials = sc.get("diff_partials", int(_m().diffuse_partials_len(m, C, r_hi - r_lo)), torch.float64, mm.device)
    totals = sc.get("diff_totals", 2 * m, torch.float64, mm.device)
    wts = hip_ops._diff_weights(w)
    side = torch.cuda.Stream(priority=0)

    def stencil(stream):
        _m().diffuse_stencil(m, R, C, r_lo, r_hi, wrap, _p(mm), _p(tmp), _p(wts[1]), _p(wts[2]), 0, 0, _p(partials),
                             _p(totals), _mdt(mm), 0, stream, 0, 1.0)

    def activity():
        hip_ops.enzymatic_activity(w)

    def timed(fn):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) * 1e3 / iters, 1)

    main_s = torch.cuda.current_stream().cuda_stream

    def both():
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        stencil(side.cuda_stream)
        activity()
        ev2 = torch.cuda.Event()
        ev2.record(side)
        torch.cuda.current_stream().wait_event(ev2)

    out = {"size": size, "cells": w.n_cells}
    for _ in range(2):
        out["activity_us"] = timed(activity)
        out["stencil_us"] = timed(lambda: stencil(main_s))
        out["serial_us"] = timed(lambda: (stencil(main_s), activity()))
        out["concurrent_us"] = timed(both)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
