"""Neighbour exchange and small all-reduces of the strip-decomposed world.

Two implementations of one interface (``exchange`` with the rows above / below, in-place
``allreduce_``, ``native``):

* :class:`RcclComm` -- GPU ranks: a dedicated RCCL communicator driven from C++
  (``csrc/hip/comm.hip``). Every call enqueues RCCL work on the current HIP stream, ordered with
  the kernels around it, with no host synchronisation and no torch.distributed work objects. The
  communicator is created over a unique id broadcast through the bootstrap process group; the RCCL
  library is the one PyTorch loaded.
* :class:`TorchComm` -- ``torch.distributed`` point-to-point / all-reduce: gloo for CPU worlds
  (tests, rehearsals); device tensors over gloo (several ranks sharing one GPU) are staged through
  host memory.

Peers are ranks of the strip ring: ``up`` owns the rows above this rank's strip, ``down`` the rows
below (the torus wraps, so with two ranks ``up == down``).
"""
from __future__ import annotations

import atexit
import datetime
import os
import weakref

import torch
import torch.distributed as dist

_LIVE: "weakref.WeakSet" = weakref.WeakSet()
# fail-stop bound of every blocking wait on a peer (seconds): a rank whose neighbour died raises
# instead of hanging (RCCL: guarded stream waits, gloo: work timeouts)
TIMEOUT_S = float(os.environ.get("MS_COMM_TIMEOUT_S", "300"))


class CommError(RuntimeError):
    """A peer failed or did not answer within ``MS_COMM_TIMEOUT_S``; the communicators of this
    process are aborted (the job is fail-stop: restart from a checkpoint)."""


def guarded_sync(event: int = 0) -> bool:
    """Wait for the current HIP stream (or only for the native ``event`` handle, see
    magicsoup_amd.ops.streams.NEvent) while polling every live RCCL communicator of this process
    for asynchronous errors, with the :data:`TIMEOUT_S` bound. On a failure all communicators are
    aborted and :class:`CommError` is raised. Called before the host synchronisations of a
    decomposed world's step (magicsoup_amd.ops.hip_ops.wait_count).

    Returns False, without waiting, when no communicator is live (all closed, aborted or
    collected): the caller then waits for the stream / event itself."""
    live = [c for c in list(_LIVE) if getattr(c, "handle", 0)]
    if not live:
        return False
    m = live[0]._m
    why = m.rccl_guarded_wait([c.handle for c in live], live[0]._stream(), TIMEOUT_S, event)
    if why:
        for c in live:
            c.handle = 0  # aborted by the wait
        raise CommError(f"communication failed ({why}): a peer rank died or stalled")
    return True


@atexit.register
def _close_all() -> None:
    """Destroy native communicators before interpreter / library teardown (their proxy threads
    must not outlive the HIP runtime). Never blocks past :data:`TIMEOUT_S`: a communicator with an
    error, or a device that does not drain, is aborted instead."""
    for c in list(_LIVE):
        try:
            c.close()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass

_OPS = {"sum": 0, "max": 1, "min": 2}
_DT = {torch.int32: 0, torch.float32: 1, torch.float64: 2, torch.int64: 3}


def _nbytes(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.numel() * t.element_size()


class TorchComm:
    """torch.distributed exchanges (``stage``: device tensors over gloo go through host copies).

    ``tagless`` (off by default; on with ``MS_COMM_TAGLESS=1`` or ``tagless=True``) reproduces the matching contract of
    :class:`RcclComm`: every point-to-point op uses tag 0 and the four ops are posted in exactly the
    order ``rccl_exchange`` posts them (send up, send down, receive from down, receive from up,
    ``csrc/hip/comm.hip``), so between two ranks sends and receives match by issue order alone,
    as in RCCL. The tagged mode (up-bound messages tag 0, down-bound tag 1) would hide a protocol
    whose correctness depends on that order; running the multi-rank tests in both modes pins the
    RCCL contract on CPU (``tests/test_distributed.py``)."""

    native = False

    def __init__(self, group, rank: int, size: int, stage: bool, tagless: bool | None = None):
        self.group, self.rank, self.size, self.stage = group, rank, size, stage
        self.tagless = os.environ.get("MS_COMM_TAGLESS", "0") == "1" if tagless is None else bool(tagless)
        glob = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
        self.up = glob((rank - 1) % size)
        self.down = glob((rank + 1) % size)

    def exchange(self, to_up, to_down, from_down, from_up) -> None:
        """``to_up`` arrives at the upper neighbour as its ``from_down``, ``to_down`` at the lower one
        as its ``from_up``. ``None`` (or an empty tensor) skips an op; the peer skips the matching one."""
        to_up, to_down, from_down, from_up = (None if t is None or t.numel() == 0 else t
                                              for t in (to_up, to_down, from_down, from_up))
        if self.size == 1:  # our own up / down neighbour (one-rank strip ring): local copies
            if from_down is not None:
                from_down.copy_(to_up.view(from_down.shape))
            if from_up is not None:
                from_up.copy_(to_down.view(from_up.shape))
            return
        if self.stage:
            h = [None if t is None else t.cpu() for t in (to_up, to_down)]
            r = [None if t is None else torch.empty(t.shape, dtype=t.dtype) for t in (from_down, from_up)]
            self._p2p(h[0], h[1], r[0], r[1])
            for dst, src in zip((from_down, from_up), r):
                if dst is not None:
                    dst.copy_(src)
            return
        self._p2p(to_up, to_down, from_down, from_up)

    @staticmethod
    def _wait(work) -> None:
        try:
            work.wait(datetime.timedelta(seconds=TIMEOUT_S))
        except RuntimeError as e:  # gloo: timeout or a closed connection (peer died)
            raise CommError(f"communication failed: {e}") from e

    def _p2p(self, to_up, to_down, from_down, from_up) -> None:
        ops = []
        g = self.group
        t_dn = 0 if self.tagless else 1  # (tagless: matched by issue order, like RCCL)
        if to_up is not None:
            ops.append(dist.P2POp(dist.isend, to_up, self.up, g, 0))
        if to_down is not None:
            ops.append(dist.P2POp(dist.isend, to_down, self.down, g, t_dn))
        if from_down is not None:
            ops.append(dist.P2POp(dist.irecv, from_down, self.down, g, 0))
        if from_up is not None:
            ops.append(dist.P2POp(dist.irecv, from_up, self.up, g, t_dn))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                self._wait(req)

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> None:
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        if self.stage:
            h = t.cpu()
            self._wait(dist.all_reduce(h, op=rop, group=self.group, async_op=True))
            t.copy_(h)
        else:
            self._wait(dist.all_reduce(t, op=rop, group=self.group, async_op=True))

    def close(self) -> None:
        pass


def _rccl_path() -> str:
    return os.environ.get("MS_RCCL_LIB") or os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


class RcclComm:
    """Native RCCL communicator over the ranks of ``group`` (collective constructor)."""

    native = True

    def __init__(self, group, rank: int, size: int, device):
        from magicsoup_amd.ops import native

        self._m = m = native.hip()
        self.version = m.rccl_load(_rccl_path())
        self.rank, self.size = rank, size
        self.up, self.down = (rank - 1) % size, (rank + 1) % size
        uid = [m.rccl_unique_id() if rank == 0 else None]
        if size > 1:
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(uid, src=src, group=group)
        with torch.cuda.device(torch.device(device)):
            self.handle = m.rccl_init(uid[0], size, rank)
        _LIVE.add(self)
        from magicsoup_amd.ops import hip_ops

        if not hip_ops._GUARD:
            hip_ops._GUARD.append(guarded_sync)
        self._raw_stream = torch._C._cuda_getCurrentRawStream
        self._cur_device = torch._C._cuda_getDevice

    def _stream(self) -> int:
        return self._raw_stream(self._cur_device())

    def exchange(self, to_up, to_down, from_down, from_up) -> None:
        p = [0 if t is None else t.data_ptr() for t in (to_up, to_down, from_down, from_up)]
        n = [_nbytes(t) for t in (to_up, to_down, from_down, from_up)]
        for t in (to_up, to_down, from_down, from_up):
            if t is not None and not t.is_contiguous():
                raise ValueError("RcclComm.exchange: buffers must be contiguous")
        self._m.rccl_exchange(self.handle, self.up, self.down, p[0], n[0], p[1], n[1], p[2], n[2], p[3], n[3],
                              self._stream())

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> None:
        if not t.is_contiguous():
            raise ValueError("RcclComm.allreduce_: tensor must be contiguous")
        self._m.rccl_allreduce(self.handle, t.data_ptr(), t.numel(), _DT[t.dtype], _OPS[op], self._stream())

    def check(self) -> None:
        """Raise if the communicator reported an asynchronous error (e.g. a peer died)."""
        err = self._m.rccl_async_error(self.handle)
        if err:
            raise RuntimeError(f"RCCL communicator error: {err}")

    def close(self) -> None:
        """Destroy the communicator (collective: every rank closes at the same point). If the
        communicator reported an error, or the device does not drain within :data:`TIMEOUT_S`
        (a peer died mid-exchange), it is aborted instead, so exit never hangs."""
        h = getattr(self, "handle", 0)
        if not h:
            return
        if self._m.rccl_async_error(h):
            self.handle = 0
            self._m.rccl_destroy(h, True)
            return
        why = self._m.rccl_guarded_wait([h], self._stream(), TIMEOUT_S)
        self.handle = 0
        if why:
            return  # aborted by the wait
        torch.cuda.synchronize()
        self._m.rccl_destroy(h, False)


def make_comm(group, rank: int, size: int, device):
    """RCCL for GPU ranks in an nccl process group (unless ``MS_NATIVE_COMM=0``), else torch.distributed."""
    dev = torch.device(device)
    backend = dist.get_backend(group)
    if dev.type == "cuda" and backend == "nccl" and os.environ.get("MS_NATIVE_COMM", "1") != "0":
        return RcclComm(group, rank, size, dev)
    return TorchComm(group, rank, size, stage=dev.type == "cuda" and backend == "gloo")
