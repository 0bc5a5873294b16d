"""Early diffusion stencil (hip_ops.spec_diffuse_issue, opt-in): kill_cells starts the stencil of the
following "degrade, then diffuse" on a side stream; diffuse_molecules adopts it only when nothing in
between read or wrote the map. Every case must give the map / cell molecules of a world that runs the
stencil in diffuse_molecules, bit for bit (GPU only)."""
import copy

import pytest
import torch

import magicsoup_amd as ms
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY
from magicsoup_amd.ops import hip_ops
from tests.conftest import gen_genomes

pytestmark = pytest.mark.gpu


def _pair(n=400, size=96, seed=7):
    ms.set_seed(seed)
    torch.manual_seed(seed)
    w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=seed)
    w.spawn_cells(gen_genomes(n, 500))
    w.enzymatic_activity()
    ref = copy.deepcopy(w)
    w.__dict__["_early_diffuse"] = True  # (off by default)
    ref.__dict__["_early_diffuse"] = False
    return w, ref


def _kill_mask(w):
    atp = CHEMISTRY.molname_2_idx["ATP"]
    return w.cell_molecules[:, atp] < 2.0


def _same(a, b):
    torch.cuda.synchronize()
    assert a.n_cells == b.n_cells
    assert torch.equal(a.cell_molecules, b.cell_molecules)
    assert torch.equal(a.molecule_map, b.molecule_map)


def _run(w, between):
    """kill -> recombinate -> mutate -> [between] -> degrade -> diffuse (no division: its placement
    order is not deterministic, and it never touches the map)"""
    w.kill_cells(_kill_mask(w))
    w.recombinate_cells()
    w.mutate_cells()
    between(w)
    w.degrade_molecules()
    w.diffuse_molecules()
    w.increment_cell_lifetimes()


def test_adopted_stencil_matches_the_regular_one(monkeypatch):
    adopted = []
    orig = hip_ops._spec_diffuse_adopt

    def spy(world):
        out = orig(world)
        adopted.append(out)
        return out

    monkeypatch.setattr(hip_ops, "_spec_diffuse_adopt", spy)
    w, ref = _pair()
    for _ in range(3):
        for x in (w, ref):
            _run(x, lambda _: None)
            x.enzymatic_activity()
        _same(w, ref)
    assert adopted == [True, True, True]


def _read_map(w):
    float(w.molecule_map.sum())


def _write_map(w):
    mm = w.molecule_map
    mm[:, 3:9, 5:40] += 1.5


def _degrade_twice(w):
    w.degrade_molecules()


def _activity(w):
    w.enzymatic_activity()


def _spawn(w):
    w.spawn_cells(gen_genomes(20, 300))


@pytest.mark.parametrize("between", [_read_map, _write_map, _degrade_twice, _activity, _spawn])
def test_voided_stencil_falls_back_exactly(between):
    w, ref = _pair()
    if between is _spawn:
        torch.manual_seed(11)
        ms.set_seed(11)
        _run(w, between)
        torch.manual_seed(11)
        ms.set_seed(11)
        _run(ref, between)
    else:
        _run(w, between)
        _run(ref, between)
    assert w.__dict__.get("_spec_diff") is None
    _same(w, ref)


def test_diffuse_without_degrade_and_loops_without_diffusion():
    w, ref = _pair()
    for x in (w, ref):
        x.kill_cells(_kill_mask(x))
        x.diffuse_molecules()  # no degradation in between: the early stencil fused one
    _same(w, ref)
    # a loop that never diffuses: speculation backs off after two voided stencils
    for _ in range(4):
        for x in (w, ref):
            x.kill_cells(_kill_mask(x))
            x.enzymatic_activity()
    assert w.__dict__.get("_spec_diff_miss", 0) >= 2
    for x in (w, ref):
        x.degrade_molecules()
        x.diffuse_molecules()
    _same(w, ref)


def test_bench_steps_with_divisions_keep_invariants():
    import bench

    atp = CHEMISTRY.molname_2_idx["ATP"]
    ms.set_seed(3)
    torch.manual_seed(3)
    w = ms.World(chemistry=CHEMISTRY, map_size=128, device="cuda", seed=3)
    w.__dict__["_early_diffuse"] = True
    w.spawn_cells(gen_genomes(2000, 500))
    for _ in range(6):
        bench.step(w, 2000, 500, atp)
    torch.cuda.synchronize()
    w.check_invariants(where="bench steps")
    assert w.__dict__.get("_spec_diff_miss", 0) == 0
    assert torch.isfinite(w.molecule_map).all() and (w.molecule_map >= 0).all()
