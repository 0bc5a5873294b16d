"""Host-side sizing rules of the device genome pipeline (ops/genome_pipeline.py): the total-length
bound its expected counts use and the per-call scratch bound."""
from types import SimpleNamespace

from magicsoup_amd.ops import genome_pipeline as gp


def _world(top_ub: int):
    return SimpleNamespace(_genomes=SimpleNamespace(top_ub=top_ub))


def test_total_length_bound_takes_the_smaller_of_rows_and_pool():
    # a typical population: n genomes at the length bound exceed the pool's used bytes
    assert gp._nt(_world(30_000_000), 50_000, 1024) == 30_000_000
    # a long evolving run: one giant genome raises the bound, the pool stays small
    assert gp._nt(_world(120_000_000), 50_000, 1_000_000) == 120_000_000
    # a fresh pool smaller than n x L is the bound; a negative / empty bound is 0
    assert gp._nt(_world(5_000), 10, 1024) == 5_000
    assert gp._nt(_world(-1), 10, 1024) == 0
    assert gp._nt(_world(10**12), 10, 1024) == 10 * 1024


def test_scratch_bound(monkeypatch):
    monkeypatch.setattr(gp, "_token_p", lambda world: 64)
    w = _world(0)
    # the default bound: short length bounds skip the size calls
    assert gp._blob_ok(w, 4096, lambda: 1 / 0)
    monkeypatch.setattr(gp, "_BLOB_MAX", 1000)
    assert gp._blob_ok(w, 4096, lambda: [400, 600])
    assert not gp._blob_ok(w, 4096, lambda: [400, 601])
    assert gp._blob_ok(w, 4096, lambda: [])
