"""The README walkthrough of the reference (README.md:45-115) as a runnable example.

A 4-molecule chemistry with one reaction (CO2 + NADPH <-> formiat + NADP, -90 kJ), 100 random
500 bp genomes on a 128^2 map, and a loop of enzymatic activity, formiat-dependent killing and
replication, mutation / recombination and diffusion. This is the BASELINE "plumbing" config; it
runs on the CPU host core or on the GPU.

    python -m magicsoup_amd.examples.readme --steps 100 --device cpu
"""
from __future__ import annotations

import argparse

import torch

import magicsoup_amd as ms

NADPH = ms.Molecule("NADPH", 200 * 1e3)
NADP = ms.Molecule("NADP", 100 * 1e3)
FORMIAT = ms.Molecule("formiat", 20 * 1e3)
CO2 = ms.Molecule("CO2", 10 * 1e3)

MOLECULES = [NADPH, NADP, FORMIAT, CO2]
REACTIONS = [([CO2, NADPH], [FORMIAT, NADP])]
CHEMISTRY = ms.Chemistry(reactions=REACTIONS, molecules=MOLECULES)


def _sample(p: torch.Tensor) -> torch.Tensor:
    """Bernoulli draw per cell -> boolean mask (stays on the device)."""
    return torch.bernoulli(p.clamp(0.0, 1.0)).bool()


def kill_cells(world: ms.World) -> None:
    x = world.cell_molecules[:, 2]  # formiat
    world.kill_cells(cell_idxs=_sample(0.01 / (0.01 + x)))


def replicate_cells(world: ms.World) -> None:
    x = world.cell_molecules[:, 2]
    world.divide_cells_t(_sample(x**3 / (x**3 + 20.0**3)))


def mutate_cells(world: ms.World) -> None:
    world.mutate_cells(p=1e-4)
    world.recombinate_cells(p=1e-6)


def make_world(device: str = "cpu", n_cells: int = 100, map_size: int = 128, genome_size: int = 500) -> ms.World:
    world = ms.World(chemistry=CHEMISTRY, map_size=map_size, device=device)
    world.spawn_cells(genomes=[ms.random_genome(s=genome_size) for _ in range(n_cells)])
    return world


def run(world: ms.World, n_steps: int) -> ms.World:
    for _ in range(n_steps):
        world.enzymatic_activity()
        kill_cells(world)
        replicate_cells(world)
        mutate_cells(world)
        world.diffuse_molecules()
    return world


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--device", default="cpu")
    a = ap.parse_args()
    w = run(make_world(a.device), a.steps)
    print(f"{w.n_cells} cells after {a.steps} steps; mean formiat {float(w.cell_molecules[:, 2].mean()):.3f}")


if __name__ == "__main__":
    main()
