"""Cheap stream / event plumbing for the op layer.

``torch.cuda.current_stream()``, ``torch.cuda.stream(...)`` and ``torch.cuda.Event().record()``
resolve the current device in Python on every call (~10 us each); the step issues a dozen of them
(stream joins around the deferred genome chains, the halo exchange, pending pipeline calls). These
helpers go through torch's C accessors for the current stream and through pooled native HIP events
(csrc/hip/events.hip) instead. Semantics are those of the torch calls they replace: ``on_stream`` is
``torch.cuda.stream`` for a stream of the current device, :class:`NEvent` a torch.cuda.Event without
timing.
"""
from __future__ import annotations

import torch

from magicsoup_amd.ops.hip_ops import _m, _stream

_get_cur = torch._C._cuda_getCurrentStream
_set_cur = torch._C._cuda_setStream


class on_stream:
    """``with on_stream(s):`` makes ``s`` (a torch.cuda.Stream of the current device) current."""

    __slots__ = ("s", "prev")

    def __init__(self, s: torch.cuda.Stream):
        self.s = s
        self.prev = None

    def __enter__(self):
        s = self.s
        self.prev = _get_cur(s.device_index)
        _set_cur(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return s

    def __exit__(self, *exc):
        p = self.prev
        _set_cur(stream_id=p[0], device_index=p[1], device_type=p[2])
        return False


class NEvent:
    """A pooled native HIP event (no timing); returned to the pool when dropped."""

    __slots__ = ("h",)

    def __init__(self):
        self.h = _m().ev_acquire()

    def record(self, stream: int | None = None) -> "NEvent":
        """Record on the raw stream ``stream`` (default: the current stream)."""
        _m().ev_record(self.h, _stream() if stream is None else stream)
        return self

    def wait(self, stream: int | None = None) -> None:
        """Make the raw stream ``stream`` (default: the current one) wait for this event."""
        _m().ev_wait(_stream() if stream is None else stream, self.h)

    def query(self) -> bool:
        return _m().ev_query(self.h)

    def synchronize(self) -> None:
        _m().ev_sync(self.h)

    def __del__(self):
        try:
            _m().ev_release(self.h)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def join(dst: int, src: int) -> None:
    """Raw stream ``dst`` waits for everything issued to raw stream ``src`` so far."""
    _m().stream_join(dst, src)
