"""Per-operation micro-benchmarks (the workloads of the reference's ``performance/check.py``).

Wood-Ljungdahl chemistry, default 128^2 map, 10k cells with random genomes of 1000 bp +-10 %, mean
+- sd over R repetitions. Every timed region ends with ``World.synchronize()`` of the worlds involved
(deferred genome chains issued and confirmed, a speculative activity confirmed or redone, a lazy
count adopted) and a device synchronisation. The reference's
published numbers (v0.14.1, NVIDIA T4 / i5-10210U, ``performance/check.py:6-26``) are printed next to
ours.

    python performance/check.py --device cuda
    python performance/check.py --device cpu --n-cells 2000
"""
from __future__ import annotations

import json
import os
import random
import sys
import time
from argparse import ArgumentParser
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

# reference (v0.14.1) seconds: T4 GPU, CPU
REFERENCE = {
    "spawn_cells": (6.64, 7.66),
    "update_cells": (5.95, 7.17),
    "replicate_cells": (0.28, 0.37),
    "enzymatic_activity": (0.16, 4.51),
    "mutations": (0.46, 0.40),
}


def _sync(device: str, *worlds) -> None:
    """End of a timed region: every world settles its deferred work first (World.synchronize: a
    pending division count, queued genome chains and their host confirmation -- replays included --,
    a speculative activity's confirmation or redo), then the device drains."""
    for w in worlds:
        if isinstance(w, ms.World):
            w.synchronize()
    if device.startswith("cuda"):
        torch.cuda.synchronize()


def _worlds(state) -> list:
    if isinstance(state, ms.World):
        return [state]
    if isinstance(state, tuple):
        return [x for x in state if isinstance(x, ms.World)]
    return []


def _genomes(n: int, s: int, d: float = 0.1) -> list[str]:
    pop = [-int(s * d), s, int(s * d)]  # same length mix as the reference helper
    return [ms.random_genome(s + random.choice(pop)) for _ in range(n)]


_PROFILE = os.environ.get("MS_CHECK_PROFILE") == "1"  # cProfile of every timed call (stderr)


def _timed(device: str, setup, fn, reps: int, worlds=()) -> list[float]:
    """``reps`` timings of ``fn(setup())``; the clock stops after :func:`_sync` of the state's worlds
    (and of ``worlds``, for closures over a world), so no confirmation falls outside it."""
    out = []
    for _ in range(reps):
        state = setup()
        _sync(device, *_worlds(state), *worlds)
        prof = None
        if _PROFILE:
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        t0 = time.perf_counter()
        fn(state)
        _sync(device, *_worlds(state), *worlds)
        out.append(time.perf_counter() - t0)
        if prof is not None:
            import io
            import pstats

            prof.disable()
            buf = io.StringIO()
            pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(12)
            print(f"--- {1e3 * out[-1]:.1f} ms\n{buf.getvalue()}", file=sys.stderr)
    return out


def bench_spawn(device, n, s, reps):
    return _timed(device, lambda: (ms.World(chemistry=CHEMISTRY, device=device), _genomes(n, s)),
                  lambda st: st[0].spawn_cells(genomes=st[1]), reps)


def bench_update(device, n, s, reps):
    def setup():
        w = ms.World(chemistry=CHEMISTRY, device=device)
        w.spawn_cells(genomes=_genomes(n, s))
        return w

    return _timed(device, setup, lambda w: w.update_cells([(g, i) for i, g in enumerate(w.cell_genomes)]), reps)


def bench_replicate(device, n, s, reps):
    def setup():
        w = ms.World(chemistry=CHEMISTRY, device=device)
        return w, w.spawn_cells(genomes=_genomes(n, s))

    return _timed(device, setup, lambda st: st[0].divide_cells(cell_idxs=st[1]), reps)


def bench_activity(device, n, s, reps):
    def setup():
        w = ms.World(chemistry=CHEMISTRY, device=device)
        w.spawn_cells(genomes=_genomes(n, s))
        return w

    return _timed(device, setup, lambda w: w.enzymatic_activity(), reps)


def bench_mutations(device, n, s, reps):
    """The reference's list API: point mutations of all genomes, neighbour pairs, recombinations."""
    w = ms.World(chemistry=CHEMISTRY, device=device)
    genomes = _genomes(n, s)
    w.spawn_cells(genomes=genomes)
    genomes = list(w.cell_genomes)

    def fn(_):
        ms.point_mutations(seqs=genomes)
        pairs = w.get_neighbors(cell_idxs=list(range(w.n_cells)))
        ms.recombinations(seq_pairs=[(genomes[a], genomes[b]) for a, b in pairs])

    return _timed(device, lambda: None, fn, reps, worlds=(w,))


def bench_world_mutations(device, n, s, reps):
    """Device-resident equivalent: mutate_cells + recombinate_cells on the world's genome arena."""
    w = ms.World(chemistry=CHEMISTRY, device=device)
    w.spawn_cells(genomes=_genomes(n, s))

    def fn(_):
        w.mutate_cells()
        w.recombinate_cells()
        # all-cells mutate / recombinate are queued for the device genome pipeline: they are
        # issued and confirmed inside the timed region (_sync -> World.synchronize)

    return _timed(device, lambda: None, fn, reps, worlds=(w,))


PARTS = {
    "spawn_cells": bench_spawn,
    "update_cells": bench_update,
    "replicate_cells": bench_replicate,
    "enzymatic_activity": bench_activity,
    "mutations": bench_mutations,
    "world_mutations": bench_world_mutations,
}


def main() -> None:
    ap = ArgumentParser()
    ap.add_argument("--parts", nargs="*", default=list(PARTS))
    ap.add_argument("--n-cells", type=int, default=10_000)
    ap.add_argument("--genome-size", type=int, default=1_000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    print(f"{a.n_cells:,} cells, {a.genome_size:,} bp genomes, {a.reps} reps, on {a.device}", file=sys.stderr)
    PARTS["spawn_cells"](a.device, min(a.n_cells, 100), a.genome_size, 1)  # warm up (builds, caches)
    for part in a.parts:
        # each part once on a small world first (untimed): the first launch of a kernel loads its code
        # object (tens of ms for the first neighbour listing), a one-time cost of the process, not
        # of the operation; the timed reps are the reference's R full-size calls
        PARTS[part](a.device, min(a.n_cells, 200), a.genome_size, 1)
        tds = PARTS[part](a.device, a.n_cells, a.genome_size, a.reps)
        mu = sum(tds) / len(tds)
        sd = (sum((t - mu) ** 2 for t in tds) / len(tds)) ** 0.5
        # the published numbers are for 10k cells x 1000 bp only
        ref = REFERENCE.get(part) if (a.n_cells, a.genome_size) == (10_000, 1_000) else None
        ref_s = None if ref is None else (ref[0] if a.device.startswith("cuda") else ref[1])
        row = {"part": part, "mean_s": round(mu, 5), "sd_s": round(sd, 5), "device": a.device, "n_cells": a.n_cells,
               "genome_size": a.genome_size, "reference_s": ref_s,
               "speedup_vs_reference": None if ref_s is None else round(ref_s / mu, 1)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
