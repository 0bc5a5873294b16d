"""Shared test helpers.

* ``gpu`` marker: tests that need an MI355X (run with ``pytest -m gpu`` on a GPU box); everything
  else runs on CPU.
* ``gen_genomes`` / ``Retry`` mirror the reference's helpers (tests/conftest.py:6-29): random genomes
  of varying length, and a context manager tolerating a few failures of stochastic assertions.
"""
import os
import random
import sys
from contextlib import contextmanager

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from magicsoup_amd.utils.util import random_genome  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running statistical / invariant checks")
    config.addinivalue_line("markers", "one_comm_mode: multi-rank test run in the tagged comm mode only")


@pytest.fixture(params=["tagged", "tagless"])
def comm_mode(request, monkeypatch):
    """Multi-rank CPU tests run twice: with tagged gloo point-to-point ops, and ``tagless`` -- every
    op tag 0, posted in the order the RCCL exchange posts them (``MS_COMM_TAGLESS=1``,
    magicsoup_amd.parallel.comm.TorchComm) -- which pins the issue-order matching contract RCCL
    relies on. Spawned ranks inherit the environment."""
    if request.param == "tagless" and request.node.get_closest_marker("one_comm_mode"):
        pytest.skip("comm-mode independent")
    monkeypatch.setenv("MS_COMM_TAGLESS", "1" if request.param == "tagless" else "0")
    return request.param


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def gen_genomes(n: int, s: int, d: float = 0.1) -> list[str]:
    """n random genomes with lengths s, s +- d*s/2, s +- d*s."""
    pop = [-int(s * d), -int(s * d / 2), s, int(s * d / 2), int(s * d)]
    return [random_genome(s + random.choice(pop)) for _ in range(n)]


class Retry:
    """Allow up to ``n_allowed_fails`` failing assertions across repeated stochastic trials."""

    def __init__(self, n_allowed_fails: int = 0):
        self.n_allowed_fails = n_allowed_fails
        self.n_fails = 0

    @contextmanager
    def catch_assert(self, i: int):
        try:
            yield
        except AssertionError as err:
            self.n_fails += 1
            if self.n_fails > self.n_allowed_fails:
                raise AssertionError(f"Failed {self.n_fails} times after {i + 1} tries") from err

    def reset(self):
        self.n_fails = 0
