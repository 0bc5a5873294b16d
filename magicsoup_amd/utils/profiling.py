"""Tracing / timing helpers.

* roctx ranges around every World operation (visible in ``rocprofv3 --marker-trace`` timelines);
  enabled with ``MS_ROCTX=1`` so the default path pays nothing.
* :class:`PhaseTimer` — HIP-event (or wall-clock on CPU) timers per named phase, the in-library
  analogue of the reference's ``timeit`` TensorBoard helper (``performance/run_simulation.py:36-40``).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict

import torch

_roctx = None
if os.environ.get("MS_ROCTX") == "1":
    for _name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so"):
        try:
            _roctx = ctypes.CDLL(os.path.join("/opt/rocm/lib", _name))
            _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
            break
        except OSError:
            _roctx = None


def roctx_enabled() -> bool:
    return _roctx is not None


def range_push(name: str) -> None:
    if _roctx is not None:
        _roctx.roctxRangePushA(name.encode())


def range_pop() -> None:
    if _roctx is not None:
        _roctx.roctxRangePop()


@contextlib.contextmanager
def roctx_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


class PhaseTimer:
    """Accumulate per-phase times. On GPU, phases are bracketed with HIP events and resolved
    lazily (no synchronisation inside the timed loop)."""

    def __init__(self, device: str | torch.device = "cpu", sync: bool = False):
        self.gpu = torch.device(device).type == "cuda"
        # sync=True drains the device at phase boundaries, so a kernel trace can be attributed to
        # phases by timestamps (profiling only: it serialises host and device)
        self.sync = sync and self.gpu
        self._pending: list[tuple[str, object, object]] = []
        self.totals: dict[str, float] = defaultdict(float)
        self.counts: dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.sync:
            torch.cuda.synchronize()
        range_push(name)
        if self.gpu:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            try:
                yield
            finally:
                b.record()
                self._pending.append((name, a, b))
                if self.sync:
                    torch.cuda.synchronize()
                range_pop()
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self.totals[name] += (time.perf_counter() - t0) * 1e3
                self.counts[name] += 1
                range_pop()

    def summary(self) -> dict[str, dict[str, float]]:
        """{phase: {"ms_total", "ms_mean", "n"}} (synchronises pending GPU events)."""
        if self._pending:
            torch.cuda.synchronize()
            for name, a, b in self._pending:
                self.totals[name] += a.elapsed_time(b)  # type: ignore[attr-defined]
                self.counts[name] += 1
            self._pending.clear()
        return {
            k: {"ms_total": v, "ms_mean": v / max(1, self.counts[k]), "n": self.counts[k]} for k, v in self.totals.items()
        }
