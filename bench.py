"""Flagship benchmark: whole simulation steps per second.

Workload = the reference's macro benchmark loop (``performance/run_simulation.py:57-100``) at the
BASELINE.json config: Wood-Ljungdahl chemistry, 4096x4096 map, random-normal molecule map, 500 bp
random genomes, population topped up to >= 50,000 cells every step. One step:

    top up to N cells -> enzymatic_activity -> kill (ATP < 1, plus random cells so that the
    divisions that follow restore ~1.02 N: chemostat dilution) -> replicate (ATP > 5: ATP -= 4, divide)
    -> recombinate_cells -> mutate_cells -> degrade -> diffuse -> increment lifetimes

Single GPU: one ``World`` on ``cuda:0``. N GPUs: one world, domain-decomposed over N ranks, one per
GPU (``magicsoup_amd.parallel``; strong scaling of the fixed config). ``--gpus N`` launches the N ranks
itself (``torch.distributed.run`` on 127.0.0.1) unless a launcher already did (``WORLD_SIZE`` set).
Rank 0 prints one JSON line; ``value`` is steps/s of the whole job (max time over ranks); ``n_gpus``
is the size of the RCCL communicator the exchanges ran over, ``devices`` each rank's GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--map-size S] [--cells C] [--preset P]

Presets (BASELINE.json's other configs; explicit flags override a preset's values):
    flagship  4096^2, 50k cells, Wood-Ljungdahl, fp32 maps (the default; the headline metric)
    m1        16384^2, 1M cells, fp16 maps (8 GPUs: torchrun --nproc-per-node 8 bench.py --preset m1)
    wide      4096^2, 50k cells, synthetic 64 molecules / 256 reactions
    c1024     1024^2, 10k cells, synthetic 16 molecules / 32 reactions, bf16 maps
    hbm       fp16 maps, 1M cells per 16384^2, sized by utils.memory.plan to fill each GPU's HBM
"""
from __future__ import annotations

import argparse
import contextlib
import gc
import json
import math
import os
import sys
import time

import torch

BASELINE_STEPS_PER_S = 3.3  # reference, 40k cells, latest published
METRIC = "simulation steps/sec (whole node), 4096×4096 map / 50k cells, 1/2/4/8 MI355X"


PRESETS = {
    "flagship": dict(map_size=4096, cells=50_000, chemistry="wood_ljungdahl", map_dtype="fp32"),
    "m1": dict(map_size=16384, cells=1_000_000, chemistry="wood_ljungdahl", map_dtype="fp16"),
    "wide": dict(map_size=4096, cells=50_000, chemistry="synthetic:64:256", map_dtype="fp32"),
    "c1024": dict(map_size=1024, cells=10_000, chemistry="synthetic:16:32", map_dtype="bf16"),
    # the largest fp16 world (the m1 config's cell density) that fills each GPU's HBM: map side and
    # cell count from utils.memory.plan for the device's memory and the number of ranks
    "hbm": dict(chemistry="wood_ljungdahl", map_dtype="fp16"),
}


def _count(n: int) -> str:
    return f"{n // 1_000_000}M" if n % 1_000_000 == 0 else (f"{n // 1000}k" if n % 1000 == 0 else str(n))


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 60; --sustained: 200)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps first (default 20; --sustained: 200)")
    ap.add_argument("--sustained", action="store_true",
                    help="time an evolved population: steps 201-400 by default (the reference's macro run is "
                         "200 steps of an evolving population, performance/run_simulation.py:120)")
    ap.add_argument("--preset", default="flagship", choices=sorted(PRESETS))
    ap.add_argument("--map-size", type=int, default=None)
    ap.add_argument("--cells", type=int, default=None)
    ap.add_argument("--genome-size", type=int, default=500)
    ap.add_argument("--chemistry", default=None, help="wood_ljungdahl | synthetic:M:R")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--map-dtype", default=None, choices=["fp32", "bf16", "fp16"],
                    help="molecule-map storage dtype (kernels compute in fp32; default matches the reference)")
    ap.add_argument("--profile-phases", action="store_true", help="print per-phase times to stderr")
    ap.add_argument("--step-times", action="store_true", help="print each timed step's wall time to stderr "
                    "(synchronises after every step)")
    ap.add_argument("--memory-report", action="store_true", help="print the world's device bytes (utils.memory."
                    "measured) against the model (utils.memory.footprint) to stderr (default for --preset hbm)")
    ap.add_argument("--phase-sync", action="store_true", help="with --profile-phases: drain the GPU at phase "
                    "boundaries (for attributing a kernel trace to phases; slows the step)")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = 200 if a.sustained else 60
    if a.warmup is None:
        a.warmup = 200 if a.sustained else 20
    for k, v in PRESETS[a.preset].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def _chemistry(spec: str):
    if spec.startswith("synthetic"):
        from magicsoup_amd.examples.synthetic import make_chemistry

        _, m, r = spec.split(":")
        return make_chemistry(int(m), int(r), seed=0)
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    return CHEMISTRY


_LUT: dict = {}


def random_genomes(k: int, size: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    """k uniformly random genomes of ``size`` nt as a packed (bytes, lengths) batch (on device)."""
    lut = _LUT.get(str(device))
    if lut is None:
        lut = _LUT[str(device)] = torch.tensor(list(b"TCGA"), dtype=torch.uint8, device=device)
    rows = lut[torch.randint(0, 4, (k, size), device=device)]
    return rows, torch.full((k,), size, dtype=torch.int32, device=device)


# running means of divisions / starvation deaths, and the previous step's dilution (its kill and
# division counts are only read at the next step's start, when the population is known anyway)
_CHEMOSTAT = {"divided": 0, "starved": 0, "steps": 0, "excess": None, "last_d": 0, "last_s": 0}


_NULL = contextlib.nullcontext()


def step(world, n_target: int, genome_size: int, atp: int, timer=None, stats=None):
    def ph(name):
        return timer.phase(name) if timer is not None else _NULL

    def note(key, val):
        if stats is not None:
            stats[key] = stats.get(key, 0) + int(val)

    with ph("top_up"):
        n = world.n_cells
        last = world.__dict__.get("last_kill")
        if _CHEMOSTAT["excess"] is not None and last is not None:
            # the previous step's kill and divisions (issued without waiting for their counts: the
            # reference loop discards the pairs, and the counts are long on the host by now)
            n_before, after_kill = last
            d = max(0, n - after_kill)
            starved = max(0, n_before - after_kill - _CHEMOSTAT["excess"])
            first = not _CHEMOSTAT["steps"]
            _CHEMOSTAT["divided"] = d if first else (_CHEMOSTAT["divided"] + d) // 2
            _CHEMOSTAT["starved"] = starved if first else (_CHEMOSTAT["starved"] + starved) // 2
            _CHEMOSTAT["last_d"], _CHEMOSTAT["last_s"] = d, starved
            _CHEMOSTAT["steps"] += 1
            _CHEMOSTAT["excess"] = None
            note("divided", d)
            note("killed", n_before - after_kill)
        if n < n_target:
            world.spawn_cells(random_genomes(n_target - n, genome_size, world.cell_molecules.device))
            note("spawned", n_target - n)
        # chemostat dilution (see kill below): the random cells depend only on the population size
        n0 = world.n_cells
        # margin: 2 % plus three standard deviations of the step's random division / dilution counts;
        # the estimates are running means (spawned cells divide more in their first step, and a
        # last-step estimate makes the population oscillate around the target)
        # (the cautious side of the running mean and the last step: fewer divisions, more starvation
        # -- a fresh population's starvation ramps up over its first steps, and a lagging estimate
        # over-dilutes it into a top-up of thousands of random cells)
        d_est = min(_CHEMOSTAT["divided"], _CHEMOSTAT["last_d"])
        s_est = max(_CHEMOSTAT["starved"], _CHEMOSTAT["last_s"])
        margin = n_target // 50 + 3 * int(math.sqrt(d_est + 1))
        keep = n_target + margin - d_est + s_est
        excess = min(n0 - keep, n0)
    with ph("activity"):
        world.enzymatic_activity()
    with ph("kill_replicate"):
        # kill (ATP < 1) and replicate (ATP > 5: ATP -= 4, divide), performance/run_simulation.py:80-92,
        # as one call that never waits for the device (World.kill_divide_where: the threshold masks,
        # the ATP payment, the kill and the division in one native call -- the same as building the
        # masks with torch and calling kill_divide_t; the replicate mask is taken over the survivors
        # before the kill, which does not change their molecules).
        # Chemostat dilution keeps the population at the configured size (the reference loop only
        # tops up; on a 4096^2 map the population would otherwise grow ~6x within 25 steps): each
        # cell also dies with probability excess / n (drawn on the device: the chemostat needs the
        # rate, not an exact count), so that after the divisions that follow the population is back
        # at n_target plus a small margin (the previous steps' divisions and starvation deaths are
        # the estimates). The margin keeps the next step's top-up (a spawn) rare; activity always
        # runs on >= n_target cells.
        if excess > 0:
            note("diluted", excess)
        world.kill_divide_where(atp, kill_below=1.0, divide_above=5.0, divide_cost=4.0,
                                kill_fraction=excess / n0 if excess > 0 else 0.0)
        _CHEMOSTAT["excess"] = max(excess, 0)
    with ph("recombinate"):
        world.recombinate_cells()
    with ph("mutate"):
        world.mutate_cells()
    with ph("wrap_up"):
        world.degrade_molecules()
        world.diffuse_molecules()
        world.increment_cell_lifetimes()


def _prime_rare_paths(chem, device, mdt, genome_size: int) -> None:
    """Setup: run the rarely taken paths once on a small throw-away world -- the host replay after an
    arena widening, the synchronous genetics path, the parameter rebuild after a protein-dimension
    widening, the rollback of a speculative activity, a genome-pool collection. Their first launches (code-object loading of
    kernels the steady state never uses, first allocations) otherwise land in whichever timed step
    first needs them (15-29 ms steps with a short warm-up)."""
    import magicsoup_amd as ms
    from magicsoup_amd.ops import hip_ops

    w = ms.World(chemistry=chem, map_size=64, device=device, seed=1, map_dtype=mdt)
    w.spawn_cells(random_genomes(300, genome_size, device))
    atp = chem.molname_2_idx.get("ATP", 0)
    for _ in range(3):
        step(w, 300, genome_size, atp)
    idx = list(range(min(40, w.n_cells)))
    w.mutate_cells(idx, p=1e-3)  # index lists: the synchronous genetics path
    w.recombinate_cells(idx, p=1e-4)
    w.update_cells([(ms.random_genome(2 * genome_size + 100), i) for i in idx[:8]])  # long genomes: widening
    w.kinetics.increase_max_proteins(int(w.kinetics.N.size(1)) + 8)
    buf = hip_ops.save_cell_state(w)
    hip_ops.restore_cell_state(w, buf)
    w.enzymatic_activity()
    step(w, 300, genome_size, atp)
    # a genome-pool collection (dense worlds churn the pool: 256^2 / 40k collects every ~30 steps);
    # its first call loads the torch kernels it uses (~0.2 s once per process)
    w._reconcile()
    torch.cuda.synchronize()
    w._genomes.collect()
    torch.cuda.synchronize()
    del w
    _CHEMOSTAT.update(divided=0, starved=0, steps=0, excess=None, last_d=0, last_s=0)


def _self_launch(a) -> int | None:
    """``--gpus N`` (N > 1) without a launcher: start N ranks of this script under
    ``torch.distributed.run`` (one per GPU, rendezvous on 127.0.0.1) and return their exit code.
    Runs before anything touches the GPU in this process (the children initialise their own
    devices); rank 0's JSON line reaches stdout directly. A failing rank makes the launcher, and so
    this process, exit non-zero."""
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = int(sk.getsockname()[1])
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL between processes)
    env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // (2 * a.gpus))))
    return subprocess.run(cmd, env=env).returncode


def main():
    a = _args()
    rc = _self_launch(a)
    if rc is not None:
        sys.exit(rc)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size > 1 and a.gpus not in (1, world_size):
        print(f"bench.py: --gpus {a.gpus} but the launcher started {world_size} ranks; reporting "
              f"{world_size}", file=sys.stderr)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MS_VIRTUAL_STRIPS=1: one rank running the multi-rank code path (strip geometry, exchanges with
    # itself over RCCL / gloo) -- measures the protocol overhead a rank of an N-GPU job pays
    virtual = world_size == 1 and os.environ.get("MS_VIRTUAL_STRIPS") == "1"
    if virtual:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
    distributed = world_size > 1 or virtual
    n_dev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    backend = (os.environ.get("MS_DIST_BACKEND", "nccl") if n_dev else "gloo") if distributed else None
    if n_dev and local_rank >= n_dev:
        if backend != "gloo":
            # RCCL needs one rank per GPU: two ranks on one device hang or fail inside the communicator
            raise SystemExit(f"LOCAL_RANK {local_rank} >= {n_dev} visible GPUs: one rank per GPU with the nccl "
                             "backend (set MS_DIST_BACKEND=gloo to rehearse with ranks sharing GPUs)")
        local_rank %= n_dev  # gloo rehearsal on a small box: ranks share the GPUs round-robin
    if distributed:
        import torch.distributed as dist

        if torch.cuda.is_available() and backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), rank=rank,
                                    world_size=world_size)
        elif torch.cuda.is_available():
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend, rank=rank, world_size=world_size)
        else:  # CPU rehearsal of the multi-rank path
            dist.init_process_group(backend, rank=rank, world_size=world_size)
    device = f"cuda:{local_rank}" if torch.cuda.is_available() else "cpu"
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)

    import magicsoup_amd as ms
    from magicsoup_amd.utils.profiling import PhaseTimer

    chem = _chemistry(a.chemistry)
    mdt = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[a.map_dtype]
    if a.map_size is None or a.cells is None:  # the hbm preset: plan the config for this device
        from magicsoup_amd.utils import memory

        hbm = torch.cuda.get_device_properties(device).total_memory if torch.cuda.is_available() else 4 << 30
        plan = memory.plan(hbm_bytes=hbm, ranks=world_size if distributed else 1, n_molecules=len(chem.molecules),
                           map_dtype=a.map_dtype, genome_len=a.genome_size, reserve=0.2)
        a.map_size = a.map_size or plan["map_size"]
        a.cells = a.cells or plan["cells"]
        if rank == 0:
            print(json.dumps({"hbm_plan": {k: v for k, v in plan.items() if k != "per_rank"},
                              "per_rank_gib": round(plan["per_rank"]["total"] / 2**30, 1)}), file=sys.stderr)
    atp = chem.molname_2_idx.get("ATP", 0)
    ms.set_seed(a.seed + rank)
    torch.manual_seed(a.seed + rank)

    if distributed:
        from magicsoup_amd.parallel import DistributedWorld

        world = DistributedWorld(chemistry=chem, map_size=a.map_size, device=device, seed=a.seed, map_dtype=mdt,
                                 strips=True)
    else:
        world = ms.World(chemistry=chem, map_size=a.map_size, device=device, seed=a.seed, map_dtype=mdt)

    t0 = time.time()
    if torch.cuda.is_available():
        # (a plain world on this rank's device: no collectives; the kernels it warms are per process)
        _prime_rare_paths(chem, device, mdt, a.genome_size)
    total = todo = a.cells // max(1, world_size if distributed else 1)
    while todo > 0:  # (batches: a multi-million-cell population's random genomes stay a few hundred MB)
        k = min(todo, 500_000)
        world.spawn_cells(random_genomes(k, a.genome_size, device))
        todo -= k
        if todo > 0 and k == total - todo:
            # the first batch fixed the protein dimension: the whole population's storage at once
            # (the bench's chemostat holds it at ~1.03x the target)
            from magicsoup_amd.utils import memory

            world.reserve_cells(int(total * 1.05), int(a.genome_size * 1.1), memory.protein_slots(a.genome_size))
    setup_s = time.time() - t0

    def sync():
        # (World.synchronize: also confirms the last step's queued genome operations on the host,
        # so their confirmation -- and any replay it triggers -- is inside the timed window)
        world.synchronize()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if distributed:
            torch.distributed.barrier()
            if torch.cuda.is_available():
                torch.cuda.synchronize()

    n_target = a.cells // world_size if distributed else a.cells
    for _ in range(a.warmup):
        step(world, n_target, a.genome_size, atp)
    sync()
    # no cyclic-GC pause inside the timed window (as timeit does); reference counting still frees
    # every per-step temporary
    gc.collect()
    gc.disable()
    timer = PhaseTimer(device, sync=a.phase_sync) if a.profile_phases else None
    t0 = time.perf_counter()
    stats = {} if a.profile_phases else None
    per_step, per_spawn = [], []
    for _ in range(a.steps):
        t1 = time.perf_counter()
        st1 = {} if a.step_times and stats is None else stats
        step(world, n_target, a.genome_size, atp, timer, st1)
        if a.step_times:
            sync()
            per_step.append(round((time.perf_counter() - t1) * 1e3, 3))
            per_spawn.append(int((st1 or {}).get("spawned", 0)) if stats is None else None)
    sync()
    gc.enable()
    if per_step and rank == 0:
        srt = sorted(per_step)
        print(json.dumps({"step_ms": per_step, "median_ms": srt[len(srt) // 2], "max_ms": srt[-1],
                          "spawned": per_spawn}), file=sys.stderr)
    if (a.memory_report or a.preset == "hbm") and torch.cuda.is_available() and rank == 0:
        from magicsoup_amd.utils import memory

        meas = memory.measured(world)
        held = meas["bytes"]
        fp = memory.footprint(a.map_size, len(chem.molecules), a.cells, a.map_dtype, a.genome_size,
                              ranks=world_size if distributed else 1)
        print(json.dumps({"memory": {"measured_gib": round(held / 2**30, 2), "model_gib": round(fp["total"] / 2**30, 2),
                                     "model_over_measured": round(fp["total"] / held, 3),
                                     "measured_kinetics_gib": round(meas["kinetics_bytes"] / 2**30, 2),
                                     "measured_molecule_map_gib": round(meas["molecule_map_bytes"] / 2**30, 2),
                                     "allocated_gib": round(torch.cuda.memory_allocated() / 2**30, 2),
                                     "reserved_gib": round(torch.cuda.memory_reserved() / 2**30, 2),
                                     "parts_gib": {k: round(v / 2**30, 2) for k, v in fp.items()
                                                   if isinstance(v, int) and v > (1 << 20)}}}), file=sys.stderr)
    dt = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
        nc = torch.tensor([world.n_cells], dtype=torch.int64, device=device)
        torch.distributed.all_reduce(nc)
        n_cells = int(nc.item())
    else:
        n_cells = world.n_cells
    ms_per_step = dt / a.steps * 1e3
    value = a.steps / dt
    # distinct devices actually used (a gloo rehearsal may put several ranks on one GPU); with RCCL,
    # the size of the communicator the exchanges ran over
    devices = [local_rank if n_dev else -1]
    comm_size = None
    if distributed:
        devices = [None] * world_size
        torch.distributed.all_gather_object(devices, local_rank if n_dev else -1)
        c = world.__dict__.get("_comm")
        comm_size = getattr(c, "size", None) if getattr(c, "native", False) else None
    n_gpus = (len({d for d in devices if d is not None and d >= 0}) if comm_size is None else comm_size) if n_dev else 0
    if rank == 0:
        if timer is not None:
            per_step = {k: v / a.steps for k, v in (stats or {}).items()}
            print(json.dumps({"phases_ms": timer.summary(), "events_per_step": per_step, "setup_s": setup_s,
                              "n_cells": n_cells}), file=sys.stderr)
        flagship = (a.map_size, a.cells, a.chemistry) == (4096, 50_000, "wood_ljungdahl")
        metric = METRIC if flagship else (f"simulation steps/sec (whole node), {a.map_size}×{a.map_size} map / "
                                          f"{_count(a.cells)} cells, {a.chemistry}, maps {a.map_dtype}")
        out = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "steps/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / BASELINE_STEPS_PER_S, 2) if flagship else None,
            "dtype": "fp32" if a.map_dtype == "fp32" else f"fp32 (maps {a.map_dtype})",
            "data": "synthetic (random 500 bp genomes, |N(10,1)| molecule map, random-init kinetics maps)",
            "config": {
                "model": f"magicsoup World, {a.chemistry} chemistry ({len(chem.molecules)} molecules /"
                f" {len(chem.reactions)} reactions)",
                "global_batch": a.cells,
                "seq_len": a.genome_size,
                "map_size": a.map_size,
                "cells_at_end": n_cells,
                "parallelism": ("strips1-virtual" if virtual else f"spatial{world_size}") if distributed else "single",
            },
        }
        if a.sustained:
            out["window"] = f"steps {a.warmup + 1}-{a.warmup + a.steps} of an evolving population"
        out["ranks"] = world_size if distributed else 1
        out["devices"] = devices
        if distributed:
            out["config"]["ranks"] = world_size
            out["config"]["backend"] = backend
            if comm_size is not None:
                out["config"]["rccl_comm_size"] = comm_size
            if backend != "nccl" or world_size > n_dev or virtual:
                out["rehearsal"] = True  # ranks share GPUs, exchange over gloo or with themselves
        print(json.dumps(out), flush=True)
    if distributed:
        world.close()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
