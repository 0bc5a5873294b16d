"""Ensemble data parallelism: independent worlds, one (or more) per GPU, no communication in the step.

The reference has no multi-device support; its typical large experiment is many independent
replicate simulations (docs/tutorials.md). On an MI355X node that maps to one process per GPU, each
running its own :class:`~magicsoup_amd.World` with a distinct seed, and only small, rare
collectives to aggregate statistics (SURVEY.md 2.4 "ensemble DP").

    ctx = Ensemble.from_env()                       # rank / world size / device from torchrun's env
    world = ms.World(chemistry=chem, map_size=1024, device=ctx.device, seed=ctx.seed(base=0))
    ...
    stats = ctx.gather_stats({"n_cells": world.n_cells})   # list over ranks (on every rank)
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

_SEED_STRIDE = 1_000_003


@dataclass
class Ensemble:
    rank: int
    world_size: int
    device: str
    group: object = None

    @classmethod
    def from_env(cls, backend: str | None = None) -> "Ensemble":
        """Initialise (if needed) the default process group from RANK / WORLD_SIZE / MASTER_*.
        backend: ``nccl`` (RCCL) when a GPU is present, else ``gloo``. A single process without the
        torchrun environment is an ensemble of one."""
        if dist.is_initialized():
            ws, rank = dist.get_world_size(), dist.get_rank()
        else:
            ws = int(os.environ.get("WORLD_SIZE", "1"))
            rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        gpu = torch.cuda.is_available()
        device = f"cuda:{local % max(torch.cuda.device_count(), 1)}" if gpu else "cpu"
        if gpu:
            torch.cuda.set_device(torch.device(device))
        if ws > 1 and not dist.is_initialized():
            kw = {"device_id": torch.device(device)} if gpu else {}
            dist.init_process_group(backend or ("nccl" if gpu else "gloo"), rank=rank, world_size=ws, **kw)
        return cls(rank=rank, world_size=ws, device=device)

    def seed(self, base: int = 0) -> int:
        """Distinct, reproducible seed of this member."""
        return int(base) + _SEED_STRIDE * self.rank

    def _active(self) -> bool:
        return self.world_size > 1 and dist.is_initialized()

    def gather_stats(self, stats: dict) -> list[dict]:
        """All ranks' ``stats`` dicts (picklable values), in rank order, on every rank."""
        if not self._active():
            return [dict(stats)]
        out = [None] * self.world_size
        dist.all_gather_object(out, dict(stats), group=self.group)
        return out

    def reduce_sum(self, values: dict[str, float]) -> dict[str, float]:
        """Sums over ranks of scalar metrics (one small all-reduce)."""
        keys = sorted(values)
        t = torch.tensor([float(values[k]) for k in keys], dtype=torch.float64)
        if self._active():
            if dist.get_backend(self.group) == "nccl":
                t = t.to(self.device)
            dist.all_reduce(t, group=self.group)
        return dict(zip(keys, t.cpu().tolist()))

    def barrier(self) -> None:
        if self._active():
            dist.barrier(group=self.group)
