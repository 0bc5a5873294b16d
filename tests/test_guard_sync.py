"""hip_ops.guarded_sync falls back to a plain wait when the registered peer-failure guard finds no
live communicator (a stale pinned count after every communicator was closed)."""
from magicsoup_amd.ops import hip_ops


class _Ev:
    def __init__(self):
        self.synced = 0
        self.h = 7

    def synchronize(self):
        self.synced += 1


def test_guard_without_live_comms_still_waits(monkeypatch):
    calls = []

    def guard(h=0):
        calls.append(h)
        return False  # no live communicator: nothing waited

    monkeypatch.setattr(hip_ops, "_GUARD", [guard])
    ev = _Ev()
    hip_ops.guarded_sync(ev)
    assert calls == [7] and ev.synced == 1


def test_guard_with_live_comms_is_the_wait(monkeypatch):
    monkeypatch.setattr(hip_ops, "_GUARD", [lambda h=0: True])
    ev = _Ev()
    hip_ops.guarded_sync(ev)
    assert ev.synced == 0


def test_comm_guard_reports_no_live_comms():
    from magicsoup_amd.parallel import comm

    assert comm.guarded_sync(0) is False or len(comm._LIVE) > 0
