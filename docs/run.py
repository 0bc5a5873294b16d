"""Demo simulation that produces data for the visualisations (reference ``docs/run.py``).

Wood-Ljungdahl chemistry; cells pay ATP per step, die when ATP runs low, divide on acetyl-CoA (at a
cost), mutate every step and recombine once old. Every ``--check-every`` steps the run logs scalars
(JSON lines: cell count, mean concentration per molecule) and a cell-map frame, and with
``--save-state`` writes ``save_state`` checkpoints (``step=<i>/``). The world itself is pickled once
at the start (``World.save``), so ``World.from_file`` + ``load_state`` can replay any checkpoint.

The reference logs to TensorBoard; this writes ``scalars.jsonl`` and ``frames/cells_<step>.png``,
which ``docs/create_gif.py`` turns into a cell-growth GIF.

    python docs/run.py --device cuda --map-size 256 --n-steps 1000 --save-state
"""
from __future__ import annotations

import argparse
import datetime as dt
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

_THIS = Path(__file__).resolve().parent


def _sample(p: torch.Tensor) -> torch.Tensor:
    return torch.bernoulli(p.clamp(0.0, 1.0)).bool()


def _activity(world: ms.World, i_atp: int, i_adp: int) -> None:
    cm = world.cell_molecules
    cm[:, i_atp] -= 0.01
    cm[:, i_adp] += 0.01
    cm[:, i_atp].clamp_(min=0.0)
    world.enzymatic_activity()
    world.degrade_molecules()
    world.diffuse_molecules()
    world.increment_cell_lifetimes()


def _kill(world: ms.World, i_atp: int, k: float) -> None:
    x = world.cell_molecules[:, i_atp]
    world.kill_cells(_sample(k**7 / (k**7 + x**7)))


def _replicate(world: ms.World, i_aca: int, i_hca: int, k: float, cost: float = 2.0) -> None:
    x = world.cell_molecules[:, i_aca]
    want = _sample(x**5 / (x**5 + k**5)) & (x > cost)
    parents, children = world.divide_cells_t(want)
    if parents.numel():
        both = torch.cat([parents, children])
        world.cell_molecules[both, i_aca] -= cost / 2
        world.cell_molecules[both, i_hca] += cost / 2


def _mutate(world: ms.World, old: int = 10) -> None:
    world.mutate_cells()
    world.recombinate_cells(cell_idxs=torch.nonzero(world.cell_lifetimes > old).flatten())


def _log(step: int, world: ms.World, out, frames: Path | None) -> None:
    n = world.map_size**2 + world.n_cells
    mm = world.molecule_map.double().sum(dim=[1, 2])
    cm = world.cell_molecules.double().sum(0) if world.n_cells else torch.zeros_like(mm)
    rec = {"step": step, "n_cells": world.n_cells}
    for i, mol in enumerate(CHEMISTRY.molecules):
        rec[mol.name] = float((mm[i] + cm[i]) / n)
    out.write(json.dumps(rec) + "\n")
    out.flush()
    if frames is not None:
        from PIL import Image

        img = (world.cell_map.to(torch.uint8) * 255).cpu().numpy()
        Image.fromarray(img, mode="L").save(frames / f"cells_{step:06d}.png")


def main(a: argparse.Namespace) -> Path:
    rundir = Path(a.rundir) if a.rundir else _THIS / "runs" / dt.datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    rundir.mkdir(parents=True, exist_ok=True)
    frames = rundir / "frames"
    frames.mkdir(exist_ok=True)
    if a.seed is not None:
        ms.set_seed(a.seed)
        torch.manual_seed(a.seed)
    world = ms.World(chemistry=CHEMISTRY, map_size=a.map_size, mol_map_init=a.init_molmap, device=a.device,
                     seed=a.seed)
    world.save(rundir=rundir)
    idx = CHEMISTRY.molname_2_idx
    world.spawn_cells([ms.random_genome(a.init_genome_size) for _ in range(a.init_n_cells)])
    with open(rundir / "scalars.jsonl", "w") as out:
        for step in range(a.n_steps):
            _activity(world, idx["ATP"], idx["ADP"])
            _kill(world, idx["ATP"], a.k_kill)
            _replicate(world, idx["acetyl-CoA"], idx["HS-CoA"], a.k_replicate)
            _mutate(world)
            if step % a.check_every == 0:
                if a.save_state:
                    world.save_state(statedir=rundir / f"step={step}")
                _log(step, world, out, frames)
    return rundir


def _args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--rundir", default=None)
    ap.add_argument("--n-steps", type=int, default=1000)
    ap.add_argument("--map-size", type=int, default=128)
    ap.add_argument("--init-n-cells", type=int, default=1000)
    ap.add_argument("--init-genome-size", type=int, default=500)
    ap.add_argument("--init-molmap", default="randn")
    ap.add_argument("--k-kill", type=float, default=0.04)
    ap.add_argument("--k-replicate", type=float, default=15.0)
    ap.add_argument("--check-every", type=int, default=10)
    ap.add_argument("--save-state", action="store_true")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--seed", type=int, default=None)
    return ap.parse_args(argv)


if __name__ == "__main__":
    print(main(_args()))
