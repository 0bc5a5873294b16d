"""Run a test body on several CPU ranks (gloo over 127.0.0.1) in spawned processes."""
from __future__ import annotations

import os
import socket
import traceback

import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _entry(rank: int, world_size: int, port: int, fn, args, errq, backend: str = "gloo"):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["OMP_NUM_THREADS"] = "2"
    torch.set_num_threads(2)
    if backend == "nccl":
        torch.cuda.set_device(rank % torch.cuda.device_count())
        dist.init_process_group("nccl", rank=rank, world_size=world_size,
                                device_id=torch.device("cuda", rank % torch.cuda.device_count()))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world_size)
    try:
        fn(rank, world_size, *args)
    except BaseException:  # noqa: BLE001 - reported to the parent
        errq.put((rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def run_ranks(fn, world_size: int = 2, *args, timeout: float = 300.0, backend: str = "gloo") -> None:
    """Run ``fn(rank, world_size, *args)`` on ``world_size`` ranks (gloo by default; ``nccl`` puts
    rank r on GPU r) in spawned processes; re-raise the first failure."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, world_size, port, fn, args, errq, backend)) for r in range(world_size)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join()
    if not errq.empty():
        rank, tb = errq.get()
        raise AssertionError(f"rank {rank} failed:\n{tb}")
    if alive:
        raise AssertionError(f"{len(alive)} rank(s) timed out")
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad:
        raise AssertionError(f"rank exit codes {bad}")
