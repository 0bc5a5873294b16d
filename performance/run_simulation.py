"""Whole-loop macro benchmark (the workload of the reference's ``performance/run_simulation.py``).

Wood-Ljungdahl chemistry, 256^2 map, 500 bp genomes, random-normal molecule map. Every step:
top up to at least --init-cells cells, enzymatic_activity, kill (ATP < 1), divide (ATP > 5, paying
4 ATP), recombinate_cells() and mutate_cells() at default rates, degrade, diffuse and increment
lifetimes; save_state every --save-every steps. The reference logs phase times and per-molecule
means to TensorBoard; here they go to a JSON-lines file (one record per step).

    python performance/run_simulation.py --device cuda --init-cells 40000 --n-steps 200
"""
from __future__ import annotations

import json
import sys
import tempfile
import time
from argparse import ArgumentParser
from contextlib import contextmanager
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402


def main() -> None:
    ap = ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--n-steps", type=int, default=200)
    ap.add_argument("--init-cells", type=int, default=1000)
    ap.add_argument("--map-size", type=int, default=256)
    ap.add_argument("--genome-size", type=int, default=500)
    ap.add_argument("--save-every", type=int, default=100)
    ap.add_argument("--out", default=None, help="JSON-lines log (default: stdout summary only)")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()

    dev = a.device
    ms.set_seed(a.seed)
    world = ms.World(chemistry=CHEMISTRY, map_size=a.map_size, device=dev, seed=a.seed)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    sync = (lambda: torch.cuda.synchronize()) if dev.startswith("cuda") else (lambda: None)
    times: dict[str, float] = {}

    @contextmanager
    def timeit(name: str):
        sync()
        t0 = time.perf_counter()
        yield
        sync()
        times[name] = time.perf_counter() - t0

    log = open(a.out, "w") if a.out else None
    statedir = Path(tempfile.mkdtemp(prefix="ms_states_"))
    totals: dict[str, float] = {}
    t_start = time.perf_counter()
    for step in range(a.n_steps):
        times.clear()
        with timeit("perStep"):
            if world.n_cells < a.init_cells:
                with timeit("spawnCells"):
                    world.spawn_cells([ms.random_genome(a.genome_size) for _ in range(a.init_cells - world.n_cells)])
            with timeit("enzymaticActivity"):
                world.enzymatic_activity()
            with timeit("killCells"):
                world.kill_cells(world.cell_molecules[:, atp] < 1.0)
            with timeit("replicateCells"):
                repl = world.cell_molecules[:, atp] > 5.0
                world.cell_molecules[:, atp] -= 4.0 * repl
                world.divide_cells_t(repl)
            with timeit("mutateCells"):
                world.recombinate_cells()
                world.mutate_cells()
            with timeit("wrapUp"):
                world.degrade_molecules()
                world.diffuse_molecules()
                world.increment_cell_lifetimes()
            if a.save_every and step % a.save_every == 0:
                with timeit("saveState"):
                    world.save_state(statedir / f"step={step}")
        for k, v in times.items():
            totals[k] = totals.get(k, 0.0) + v
        if log:
            rec = {"step": step, "n_cells": world.n_cells, **{f"Time[s]/{k}": round(v, 6) for k, v in times.items()}}
            # the reference's per-molecule means over map pixels and cells (one synchronisation)
            rec["Molecules"] = dict(zip([mol.name for mol in CHEMISTRY.molecules], world.molecule_means()))
            log.write(json.dumps(rec) + "\n")
    wall = time.perf_counter() - t_start
    summary = {
        "n_steps": a.n_steps,
        "device": dev,
        "cells_at_end": world.n_cells,
        "s_per_step": round(wall / a.n_steps, 5),
        "steps_per_s": round(a.n_steps / wall, 2),
        "mean_phase_s": {k: round(v / a.n_steps, 6) for k, v in totals.items()},
    }
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
