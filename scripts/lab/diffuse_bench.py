"""Time World.diffuse_molecules (stencil + mass correction + permeation) on the GPU for the map
storage dtypes. usage: python scripts/lab/diffuse_bench.py [--size 4096] [--iters 30]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--vec", type=int, nargs="*", default=[0], help="stencil variants (columns per lane, 0 auto) to A/B")
    ap.add_argument("--blocks", type=int, nargs="*", default=[1024], help="stencil grid sizes (0: one block per tile)")
    ap.add_argument("--pf", type=int, nargs="*", default=[-1], help="rows loaded ahead by the vector stencils (-1 auto)")
    ap.add_argument("--band", type=int, nargs="*", default=[0], help="rows per wave band of the vector stencils (0 auto)")
    ap.add_argument("--chem", default="wl", help="wl | synthetic:M:R (molecule count of the map)")
    ap.add_argument("--dtypes", nargs="*", default=["fp32", "bf16", "fp16"])
    a = ap.parse_args()
    from magicsoup_amd.ops import native

    for vec in a.vec:
        for blocks in a.blocks:
            for pf in a.pf:
                for band in a.band:
                    native.hip().set_stencil_vec(vec)
                    native.hip().set_stencil_blocks(blocks)
                    native.hip().set_stencil_prefetch(pf)
                    native.hip().set_stencil_band(band)
                    run(a, f"vec{vec}_blocks{blocks}" + (f"_pf{pf}" if pf >= 0 else "") + f"_band{band}")
    native.hip().set_stencil_vec(0)
    native.hip().set_stencil_blocks(512)
    native.hip().set_stencil_prefetch(-1)
    native.hip().set_stencil_band(0)


def run(a, tag):
    out = {}
    chem = CHEMISTRY
    if a.chem.startswith("synthetic"):
        from magicsoup_amd.examples.synthetic import make_chemistry

        _, m, r = a.chem.split(":")
        chem = make_chemistry(int(m), int(r), seed=0)
    dts = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}
    for name in a.dtypes:
        dt = dts[name]
        w = ms.World(chemistry=chem, map_size=a.size, device="cuda", seed=0, map_dtype=dt)
        for _ in range(3):
            w.degrade_molecules()
            w.diffuse_molecules()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            w.degrade_molecules()
            w.diffuse_molecules()
        e1.record()
        torch.cuda.synchronize()
        ms_it = e0.elapsed_time(e1) / a.iters
        nbytes = w.molecule_map.numel() * w.molecule_map.element_size()
        # the fused stencil reads the map once and writes it once per call (degradation and the
        # pending mass correction are applied inside it)
        out[name] = {"ms": round(ms_it, 4), "map_MB": round(nbytes / 1e6, 1),
                     "eff_TBps": round(2 * nbytes / (ms_it * 1e-3) / 1e12, 3)}
        del w
        torch.cuda.empty_cache()
    print(json.dumps({"variant": tag, "size": a.size, "n_mol": len(chem.molecules), "diffuse": out}), flush=True)


if __name__ == "__main__":
    main()
