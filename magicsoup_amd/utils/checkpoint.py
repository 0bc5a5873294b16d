"""Checkpoint / resume.

* ``save_state`` / ``load_state`` keep the reference's on-disk format (``world.py:795-878``):
  ``cell_molecules.pt``, ``cell_map.pt``, ``molecule_map.pt``, ``cell_lifetimes.pt``,
  ``cell_positions.pt``, ``cell_divisions.pt`` (``torch.save`` of the tensors) and ``cells.fasta``
  with entries ``>{idx} {label}\\n{genome}``. States from either implementation load in the other.
  Tensors are written from host copies and loaded with ``weights_only=True``.
* Optionally an ``rng_state.pt`` with the native RNG seeds is written (new; ignored by the reference).
* ``load_world_pickle`` restores :meth:`World.save` pickles, remapping tensor storages onto the
  requested device like the reference's ``_CPU_Unpickler`` (``world.py:17-33``).
"""
from __future__ import annotations

import io
import pickle
from pathlib import Path

import torch

_FILES = ("cell_molecules", "cell_map", "molecule_map", "cell_lifetimes", "cell_positions", "cell_divisions")


def save_state(world, statedir: Path) -> None:
    statedir.mkdir(parents=True, exist_ok=True)
    for name in _FILES:
        t = getattr(world, name).detach().cpu()
        if name == "molecule_map":
            t = t.to(torch.float32)  # checkpoints always hold fp32 maps, whatever the storage dtype
        torch.save(t.clone(), statedir / f"{name}.pt")
    genomes = world.cell_genomes.tolist()
    labels = world.cell_labels.tolist()
    text = "\n".join(f">{i} {lab}\n{g}" for i, (g, lab) in enumerate(zip(genomes, labels)))
    with open(statedir / "cells.fasta", "w", encoding="utf-8") as fh:
        fh.write(text)


def _parse_fasta(text: str) -> tuple[list[str], list[str]]:
    genomes, labels = [], []
    for entry in (e.strip() for e in text.split(">")):
        if not entry:
            continue
        parts = entry.split("\n")
        names = parts[0].split()
        labels.append(names[1].strip() if len(names) > 1 else "")
        genomes.append(parts[1] if len(parts) > 1 else "")
    return genomes, labels


def load_state(world, statedir: Path, ignore_cell_params: bool = False) -> None:
    if world.n_cells > 0:
        world.kill_cells()
    dev = torch.device(world.device)

    def ld(name):
        return torch.load(statedir / f"{name}.pt", map_location=dev, weights_only=True)

    with open(statedir / "cells.fasta", "r", encoding="utf-8") as fh:
        genomes, labels = _parse_fasta(fh.read())
    n = len(genomes)
    cell_map = ld("cell_map").bool()
    world.molecule_map = ld("molecule_map").to(torch.float32).contiguous()
    world.cell_map = cell_map
    world.n_cells = 0
    world._grow(n)
    world.cell_molecules[:] = ld("cell_molecules").float()
    world.cell_lifetimes[:] = ld("cell_lifetimes").int()
    world.cell_positions[:] = ld("cell_positions").int()
    world.cell_divisions[:] = ld("cell_divisions").int()
    world._genomes.clear()
    world._labels.clear()
    world._genomes.append_strings(genomes)
    world._labels.append_strings(labels)
    if not ignore_cell_params and n > 0:
        world._update_params_rows(torch.arange(n, device=dev))


class _MapLocationUnpickler(pickle.Unpickler):
    """Load tensor storages of our own world pickles onto ``map_location``."""

    def __init__(self, fh, map_location):
        super().__init__(fh)
        self._loc = map_location

    def find_class(self, module, name):
        if module == "torch.storage" and name == "_load_from_bytes":
            loc = self._loc
            return lambda b: torch.load(io.BytesIO(b), map_location=loc, weights_only=False)
        return super().find_class(module, name)


def load_world_pickle(path: Path, device: str | None = None):
    loc = device if device is not None else ("cuda" if torch.cuda.is_available() else "cpu")
    with open(path, "rb") as fh:
        world = _MapLocationUnpickler(fh, loc).load()
    if device is not None and str(world.device) != str(device):
        world.to(device)
    return world
