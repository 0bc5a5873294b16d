"""World behaviours on the CPU path (reference tests/fast/test_world.py). The GPU path is checked
against this one in tests/test_gpu_kernels.py."""
import tempfile
from pathlib import Path

import numpy as np
import pytest
import torch

import magicsoup_amd as ms
from magicsoup_amd.examples.wood_ljungdahl import MOLECULES


def _chem(mols=None, reactions=()):
    return ms.Chemistry(molecules=list(mols or MOLECULES), reactions=list(reactions))


def _diffuse_oracle(x: np.ndarray, rate: float) -> np.ndarray:
    """3x3 toroidal stencil with the reference's weights (world.py:948-971), mass-corrected, >= 0."""
    rate = min(abs(rate), 1.0)
    if rate == 0:
        return x.copy()
    d = 1 / rate
    a = 1 / (d + 8)
    b = d * a
    b = b + 1.0 - (8 * a + b)
    nb = sum(np.roll(np.roll(x, i, 0), j, 1) for i in (-1, 0, 1) for j in (-1, 0, 1) if (i, j) != (0, 0))
    y = b * x + a * nb
    y += (x.sum() - y.sum()) / x.size
    return np.maximum(y, 0.0)


# --------------------------------------------------------------------------------------------- physics
def test_diffusion_point_sources():
    m0 = ms.Molecule("WTdiffA", 10, diffusivity=0.0)
    m1 = ms.Molecule("WTdiffB", 10, diffusivity=0.5)
    w = ms.World(chemistry=_chem([m0, m1]), map_size=5)
    mm = torch.zeros(2, 5, 5)
    mm[0, 1, 3] = 2.0
    mm[1, 0, 0] = 1.0
    mm[1, 4, 2] = 1.0
    w.molecule_map = mm
    w.diffuse_molecules()
    out = w.molecule_map
    assert out.shape == (2, 5, 5)
    assert torch.equal(out[0], mm[0])  # diffusivity 0: unchanged
    # rate 0.5: a = 0.1 to each neighbour, b = 0.2 stays
    exp = torch.zeros(5, 5)
    for x, y in ((0, 0), (4, 2)):
        for dx in (-1, 0, 1):
            for dy in (-1, 0, 1):
                exp[(x + dx) % 5, (y + dy) % 5] += 0.2 if dx == dy == 0 else 0.1
    assert torch.allclose(out[1], exp, atol=1e-7)


@pytest.mark.parametrize("size", [3, 8, 33])
@pytest.mark.parametrize("rate", [0.01, 0.3, 1.0])
def test_diffusion_matches_numpy_oracle(size, rate):
    mol = ms.Molecule(f"WTdiff{size}_{int(rate * 100)}", 10, diffusivity=rate)
    w = ms.World(chemistry=_chem([mol]), map_size=size)
    x = w.molecule_map[0].double().numpy().copy()
    for _ in range(3):
        w.diffuse_molecules()
        x = _diffuse_oracle(x, rate)
    assert np.allclose(w.molecule_map[0].numpy(), x, rtol=1e-5, atol=1e-5)
    assert abs(w.molecule_map[0].double().sum().item() - x.sum()) / x.sum() < 1e-6


def test_degradation_scales_map_and_cells():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=5)
    w.spawn_cells([ms.random_genome(100)])
    w._mol_degrads = [0.8, 0.5]
    mm = w.molecule_map.clone()
    cm = w.cell_molecules.clone()
    w.degrade_molecules()
    assert torch.allclose(w.molecule_map[0], mm[0] * 0.8)
    assert torch.allclose(w.molecule_map[1], mm[1] * 0.5)
    assert torch.allclose(w.cell_molecules, cm * torch.tensor([0.8, 0.5]))


def test_degradation_rate_from_half_life():
    mol = ms.Molecule("WThalf", 10, half_life=4)
    w = ms.World(chemistry=_chem([mol]), map_size=4)
    before = w.molecule_map.clone()
    for _ in range(4):
        w.degrade_molecules()
    assert torch.allclose(w.molecule_map, before * 0.5, rtol=1e-5)


def test_permeation_exchanges_towards_equilibrium():
    mol = ms.Molecule("WTperm", 10, permeability=1.0)
    w = ms.World(chemistry=_chem([mol]), map_size=4, mol_map_init="zeros")
    w.spawn_cells([ms.random_genome(50)])
    x, y = w.cell_positions[0].tolist()
    w.cell_molecules[0, 0] = 6.0
    w.molecule_map[0, x, y] = 0.0
    from magicsoup_amd.ops import world_ops

    world_ops.permeate(w)
    # p = 1 / (1/1 + 1) = 0.5 of the difference moves
    assert torch.isclose(w.cell_molecules[0, 0], torch.tensor(3.0))
    assert torch.isclose(w.molecule_map[0, x, y], torch.tensor(3.0))


# --------------------------------------------------------------------------------------------- lifecycle
def test_spawn_cells_take_half_of_their_pixel():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=5)
    mm0 = w.molecule_map.clone()
    for batch in ([ms.random_genome(400) for _ in range(3)], ["", ""], [ms.random_genome(90), "", ms.random_genome(90)]):
        w.spawn_cells(genomes=batch)
        xs, ys = w.cell_positions[:, 0].long(), w.cell_positions[:, 1].long()
        assert torch.allclose(w.molecule_map[:, xs, ys], mm0[:, xs, ys] / 2)
        assert torch.allclose(w.cell_molecules.T, mm0[:, xs, ys] / 2)
    assert w.n_cells == 8
    assert int(w.cell_map.sum()) == 8
    assert len(set(w.cell_labels)) == 8
    assert (w.cell_lifetimes == 0).all() and (w.cell_divisions == 0).all()


def test_spawn_more_cells_than_pixels():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=3)
    idxs = w.spawn_cells([ms.random_genome(50) for _ in range(20)])
    assert len(idxs) == 9 and w.n_cells == 9
    assert bool(w.cell_map.all())
    assert w.spawn_cells([ms.random_genome(50)]) == []


def test_add_cells_keeps_their_state():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=6)
    mm0 = w.molecule_map.clone()
    genomes = [ms.random_genome(s) for s in (400, 200, 100)]
    cells = [
        ms.Cell(world=w, label="L0", genome=genomes[0], int_molecules=torch.tensor([1.5, 0.5])),
        ms.Cell(world=w, label="L1", genome=genomes[1], int_molecules=torch.tensor([0.25, 2.0])),
        ms.Cell(world=w, label="L2", genome=genomes[2], int_molecules=torch.tensor([3.0, 0.0]), n_steps_alive=7,
                n_divisions=2),
    ]
    assert w.add_cells(cells[:2]) == [0, 1]
    assert w.add_cells(cells[2:]) == [2]
    xs, ys = w.cell_positions[:, 0].long(), w.cell_positions[:, 1].long()
    assert torch.equal(w.molecule_map[:, xs, ys], mm0[:, xs, ys])  # no pickup
    assert torch.equal(w.cell_molecules, torch.tensor([[1.5, 0.5], [0.25, 2.0], [3.0, 0.0]]))
    assert w.cell_lifetimes.tolist() == [0, 0, 7]
    assert w.cell_divisions.tolist() == [0, 0, 2]
    assert list(w.cell_genomes) == genomes
    assert list(w.cell_labels) == ["L0", "L1", "L2"]


def test_divide_cells_split_and_inherit():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=6)
    idxs = w.spawn_cells([ms.random_genome(500) for _ in range(3)])
    before = w.cell_molecules.clone()
    pairs = w.divide_cells(idxs)
    assert sorted(p for p, _ in pairs) == [0, 1, 2]
    assert sorted(c for _, c in pairs) == [3, 4, 5]
    assert int(w.cell_map.sum()) == 6
    for p, c in pairs:
        assert torch.allclose(w.cell_molecules[p], before[p] / 2)
        assert torch.equal(w.cell_molecules[c], w.cell_molecules[p])
        assert w.cell_genomes[p] == w.cell_genomes[c]
        assert w.cell_labels[p] == w.cell_labels[c]
        assert torch.equal(w.kinetics.N[p], w.kinetics.N[c])
        px, py = w.cell_positions[p].tolist()
        cx, cy = w.cell_positions[c].tolist()
        assert ms.dist_1d(px, cx, 6) <= 1 and ms.dist_1d(py, cy, 6) <= 1


def test_divide_on_full_maps():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=2)
    idxs = w.spawn_cells([ms.random_genome(300) for _ in range(2)])
    assert len(w.divide_cells(idxs)) == 2
    assert int(w.cell_map.sum()) == 4
    assert w.divide_cells(idxs) == []
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=3)
    w.spawn_cells([ms.random_genome(300) for _ in range(9)])
    assert w.divide_cells(list(range(9))) == []


def test_divisions_and_lifetimes_after_division():
    w = ms.World(chemistry=_chem(), map_size=16)
    w.spawn_cells([ms.random_genome(300) for _ in range(2)])
    w.cell_divisions[0] = 3
    w.cell_divisions[1] = 8
    w.cell_lifetimes[0] = 4
    w.cell_lifetimes[1] = 9
    w.divide_cells([1])
    assert w.cell_divisions.tolist() == [3, 9, 9]
    assert w.cell_lifetimes.tolist() == [4, 0, 0]
    w.increment_cell_lifetimes()
    assert w.cell_lifetimes.tolist() == [5, 1, 1]


def test_move_cells_keep_state():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=32)
    idxs = w.spawn_cells([ms.random_genome(300) for _ in range(4)])
    mols, labels, genomes = w.cell_molecules.clone(), list(w.cell_labels), list(w.cell_genomes)
    for _ in range(4):
        old = w.cell_positions.clone()
        w.move_cells(idxs)
        assert int(w.cell_map.sum()) == 4
        assert torch.equal(w.cell_molecules, mols)
        assert list(w.cell_labels) == labels and list(w.cell_genomes) == genomes
        for i in idxs:
            (ox, oy), (nx, ny) = old[i].tolist(), w.cell_positions[i].tolist()
            assert (ox, oy) != (nx, ny)
            assert ms.dist_1d(ox, nx, 32) <= 1 and ms.dist_1d(oy, ny, 32) <= 1
            assert bool(w.cell_map[nx, ny])


def test_reposition_cells():
    w = ms.World(chemistry=_chem(), map_size=64)
    w.spawn_cells([ms.random_genome(300) for _ in range(3)])
    c0 = [w.get_cell(by_idx=i) for i in range(3)]
    w.reposition_cells([0, 2])
    c1 = [w.get_cell(by_idx=i) for i in range(3)]
    assert c1[0].position != c0[0].position and c1[2].position != c0[2].position
    assert c1[1].position == c0[1].position
    for a, b in zip(c0, c1):
        assert torch.equal(a.int_molecules, b.int_molecules)
        assert (a.genome, a.label) == (b.genome, b.label)
    assert int(w.cell_map.sum()) == 3


def test_molecules_are_conserved_by_spawn_divide_kill():
    w = ms.World(chemistry=_chem(), map_size=64)
    total = lambda: w.molecule_map.double().sum(dim=[1, 2]) + w.cell_molecules.double().sum(dim=0)  # noqa: E731
    exp = total()
    idxs = w.spawn_cells([ms.random_genome(500) for _ in range(500)])
    assert torch.allclose(total(), exp, rtol=1e-6)
    pairs = w.divide_cells(idxs)
    assert torch.allclose(total(), exp, rtol=1e-6)
    w.kill_cells(idxs + [c for _, c in pairs])
    assert torch.allclose(total(), exp, rtol=1e-6)
    assert w.n_cells == 0 and int(w.cell_map.sum()) == 0


def test_indices_stay_consistent():
    w = ms.World(chemistry=_chem(), map_size=64)
    idxs = w.spawn_cells([ms.random_genome(1000) for _ in range(600)])
    n0 = w.n_cells
    assert n0 == 600 and len(w.cell_genomes) == n0 and len(set(w.cell_labels)) == n0
    pairs = w.divide_cells(idxs)
    n1 = w.n_cells
    assert n1 == n0 + len(pairs)
    assert {p for p, _ in pairs} <= set(idxs) and not {c for _, c in pairs} & set(idxs)
    assert len(set(w.cell_labels)) == n0
    # kill parents: children shift down to the front, keeping their order and genomes
    child_genomes = [w.cell_genomes[c] for _, c in pairs]
    w.kill_cells(idxs)
    assert w.n_cells == len(pairs)
    assert list(w.cell_genomes) == child_genomes
    assert int(w.cell_map.sum()) == w.n_cells
    assert w.kinetics.N.size(0) == w.n_cells
    w.kill_cells(list(range(w.n_cells)))
    assert w.n_cells == 0 and int(w.cell_map.sum()) == 0


def test_kill_removes_params_rows():
    w = ms.World(chemistry=_chem(), map_size=16)
    w.spawn_cells([ms.random_genome(800) for _ in range(10)])
    N = w.kinetics.N.clone()
    w.kill_cells([1, 4, 5])
    keep = [0, 2, 3, 6, 7, 8, 9]
    assert torch.equal(w.kinetics.N, N[keep])


def test_get_cell_by_index_and_position():
    w = ms.World(chemistry=_chem(MOLECULES[:2]), map_size=5)
    w.spawn_cells([ms.random_genome(300) for _ in range(3)])
    pos = tuple(w.cell_positions[2].tolist())
    c = w.get_cell(by_position=pos)
    assert c.idx == 2 and c.position == pos
    assert c.genome == w.cell_genomes[2] and c.label == w.cell_labels[2]
    free = [(x, y) for x in range(5) for y in range(5) if not w.cell_map[x, y]][0]
    with pytest.raises(ValueError):
        w.get_cell(by_position=free)


def test_update_cells_and_empty_genomes():
    w = ms.World(chemistry=_chem(), map_size=16)
    g0, g1, g2 = ms.random_genome(500), ms.random_genome(1000), ms.random_genome(600)
    w.spawn_cells([g0, g0])
    assert torch.equal(w.kinetics.N[0], w.kinetics.N[1])
    w.spawn_cells([g1])
    w.update_cells([(g2, 1)])
    assert list(w.cell_genomes) == [g0, g2, g1]
    w.kill_cells([0])
    assert list(w.cell_genomes) == [g2, g1]
    w.update_cells([(g0, 0), ("", 1)])
    assert list(w.cell_genomes) == [g0, ""]
    assert (w.kinetics.N[1] == 0).all() and (w.kinetics.Vmax[1] == 0).all()
    w.update_cells([("", 0)])
    assert (w.kinetics.N == 0).all()


def test_empty_proteome_cells():
    w = ms.World(chemistry=_chem(), map_size=9)
    genomes = [ms.random_genome(10), "", ms.random_genome(12)]
    w.spawn_cells(genomes)
    assert all(len(w.get_cell(by_idx=i).proteome) == 0 for i in range(3))
    w.enzymatic_activity()  # nothing to do, nothing breaks
    assert torch.isfinite(w.cell_molecules).all()


def test_neighbors_fixture():
    w = ms.World(chemistry=_chem(), map_size=7)
    pos = [(0, 0), (0, 1), (6, 6), (3, 3), (4, 4), (3, 5), (0, 6), (5, 0)]
    w.n_cells = len(pos)
    w.cell_positions = torch.tensor(pos, dtype=torch.int32)
    cm = torch.zeros(7, 7, dtype=torch.bool)
    for x, y in pos:
        cm[x, y] = True
    w.cell_map = cm

    def brute(frm, to):
        out = set()
        for a in frm:
            for b in to:
                if a == b:
                    continue
                (ax, ay), (bx, by) = pos[a], pos[b]
                if ms.dist_1d(ax, bx, 7) <= 1 and ms.dist_1d(ay, by, 7) <= 1:
                    out.add((min(a, b), max(a, b)))
        return out

    everyone = list(range(len(pos)))
    for i in everyone:
        assert set(w.get_neighbors([i], everyone)) == brute([i], everyone)
    assert set(w.get_neighbors(everyone)) == brute(everyone, everyone)
    # toroidal wrap: (0,0)-(6,6), (0,0)-(0,6), (0,6)-(6,6), (5,0)-(6,6)
    assert {(0, 2), (0, 6), (2, 6), (2, 7)} <= set(w.get_neighbors(everyone))
    assert set(w.get_neighbors([3, 4], [5])) == brute([3, 4], [5]) == {(4, 5)}
    res = w.get_neighbors([0, 3])
    assert res == sorted(res)


def test_public_tensors_are_stable_references():
    w = ms.World(chemistry=_chem(), map_size=4, mol_map_init="zeros")
    w.spawn_cells([ms.random_genome(400) for _ in range(2)])
    refs = (w.molecule_map, w.cell_molecules, w.cell_map)
    w.diffuse_molecules()
    w.enzymatic_activity()
    w.degrade_molecules()
    assert w.molecule_map is refs[0] and w.cell_molecules is refs[1] and w.cell_map is refs[2]
    w.molecule_map = torch.full_like(w.molecule_map, 2.0)
    w.cell_molecules = torch.full_like(w.cell_molecules, 2.0)
    assert float(w.molecule_map.mean()) == 2.0 and float(w.cell_molecules.mean()) == 2.0
    refs = (w.molecule_map, w.cell_molecules)
    w.diffuse_molecules()
    w.enzymatic_activity()
    assert w.molecule_map is refs[0] and w.cell_molecules is refs[1]


# --------------------------------------------------------------------------------------------- persistence
def test_save_and_load_state_roundtrip():
    mi, mj = ms.Molecule("WTsaveI", 10e3), ms.Molecule("WTsaveJ", 20e3)
    chem = ms.Chemistry(molecules=[mi, mj], reactions=[([mi], [mj])])
    w = ms.World(chemistry=chem, map_size=7)
    w.spawn_cells([ms.random_genome(500) for _ in range(3)] + [""])
    w.cell_lifetimes[1] = 5
    w.cell_divisions[2] = 2
    with tempfile.TemporaryDirectory() as d:
        w.save_state(Path(d))
        assert {p.name for p in Path(d).iterdir()} >= {"cells.fasta"}
        w2 = ms.World(chemistry=chem, map_size=7)
        w2.load_state(Path(d))
    assert torch.equal(w2.cell_map, w.cell_map)
    assert torch.equal(w2.molecule_map, w.molecule_map)
    assert torch.equal(w2.cell_molecules, w.cell_molecules)
    assert torch.equal(w2.cell_positions, w.cell_positions)
    assert w2.cell_lifetimes.tolist() == w.cell_lifetimes.tolist()
    assert w2.cell_divisions.tolist() == w.cell_divisions.tolist()
    assert list(w2.cell_genomes) == list(w.cell_genomes)
    assert list(w2.cell_labels) == list(w.cell_labels)


def test_loading_several_states_replaces_cells():
    mi, mj = ms.Molecule("WTsaveI", 10e3), ms.Molecule("WTsaveJ", 20e3)
    chem = ms.Chemistry(molecules=[mi, mj], reactions=[([mi], [mj])])
    with tempfile.TemporaryDirectory() as d:
        w = ms.World(chemistry=chem, map_size=7)
        counts = []
        for k, action in enumerate(("spawn", "spawn", "kill")):
            if action == "spawn":
                w.spawn_cells([ms.random_genome(500) for _ in range(3)])
            else:
                w.kill_cells(list(range(4)))
            w.save_state(Path(d) / f"s{k}")
            counts.append(w.n_cells)
        assert counts == [3, 6, 2]
        w = ms.World(chemistry=chem, map_size=7)
        for k in (0, 1, 2, 0):
            w.load_state(Path(d) / f"s{k}", ignore_cell_params=(k == 1))
            assert w.n_cells == counts[k] == len(w.cell_genomes) == int(w.cell_map.sum())
            assert w.kinetics.N.size(0) == counts[k]


def test_save_and_from_file_world_object():
    mi, mj = ms.Molecule("WTsaveI", 10e3), ms.Molecule("WTsaveJ", 20e3)
    chem = ms.Chemistry(molecules=[mi, mj], reactions=[([mi], [mj])])
    for size, temp in ((7, 310.0), (9, 300.0)):
        w = ms.World(chemistry=chem, map_size=size, abs_temp=temp)
        w.spawn_cells([ms.random_genome(400) for _ in range(4)])
        with tempfile.TemporaryDirectory() as d:
            w.save(rundir=Path(d))
            w2 = ms.World.from_file(rundir=Path(d))
        assert (w2.abs_temp, w2.map_size, w2.device) == (temp, size, "cpu")
        assert w2.chemistry.molecules[0] is mi and w2.chemistry.molecules[1] is mj
        assert w2.chemistry.reactions == [([mi], [mj])]
        assert w2.chemistry.mol_2_idx == {mi: 0, mj: 1}
        assert list(w2.cell_genomes) == list(w.cell_genomes)
        assert torch.equal(w2.kinetics.N, w.kinetics.N)
        assert torch.equal(w2.kinetics.Vmax, w.kinetics.Vmax)
        w2.enzymatic_activity()  # usable after restore


def test_load_without_then_with_cell_params(tmp_path):
    # reference quirk 8: a load with ignore_cell_params must still leave kinetics with
    # exactly one row per cell so that a later full load replaces cleanly
    mi, mj = ms.Molecule("LWi", 10e3), ms.Molecule("LWj", 20e3)
    chem = ms.Chemistry(molecules=[mi, mj], reactions=[([mi], [mj])])
    world = ms.World(chemistry=chem, map_size=7)
    world.spawn_cells(genomes=[ms.random_genome(s=500) for _ in range(3)])
    world.save_state(statedir=tmp_path / "s0")
    world.spawn_cells(genomes=[ms.random_genome(s=500) for _ in range(3)])
    world.save_state(statedir=tmp_path / "s1")
    assert world.n_cells == 6 and world.kinetics.N.size(0) == 6

    world = ms.World(chemistry=chem, map_size=7)
    world.load_state(statedir=tmp_path / "s0", ignore_cell_params=True)
    assert world.n_cells == 3 and len(world.cell_genomes) == 3
    assert world.kinetics.N.size(0) == 3
    world.load_state(statedir=tmp_path / "s1")
    assert world.n_cells == 6 and len(world.cell_genomes) == 6
    assert world.kinetics.N.size(0) == 6
    assert int(world.cell_map.sum()) == 6


def _evolve(w, steps):
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(steps):
        w.enzymatic_activity()
        w.kill_cells(torch.nonzero(w.cell_molecules[:, atp] < 1.0).flatten().tolist())
        w.divide_cells(torch.nonzero(w.cell_molecules[:, atp] > 3.0).flatten().tolist())
        w.recombinate_cells(p=1e-4)
        w.mutate_cells(p=1e-3)
        w.degrade_molecules()
        w.diffuse_molecules()
        w.increment_cell_lifetimes()


def test_save_load_state_resumes_rng_streams(tmp_path):
    """save_state writes rng_state.pt; load_state(restore_rng=True) restores it: save -> load -> N steps gives
    exactly what N uninterrupted steps give (placement, mutations, recombination, labels)."""
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    ms.set_seed(21)
    torch.manual_seed(21)
    w = ms.World(chemistry=CHEMISTRY, map_size=24, seed=21)
    w.spawn_cells([ms.random_genome(400) for _ in range(120)])
    _evolve(w, 2)
    w.save_state(tmp_path / "s")
    assert (tmp_path / "s" / "rng_state.pt").exists()
    _evolve(w, 3)
    w.spawn_cells([ms.random_genome(300) for _ in range(5)])
    ms.set_seed(21)
    w2 = ms.World(chemistry=CHEMISTRY, map_size=24, seed=21)  # same codon / kinetics maps
    ms.set_seed(99)  # streams that would diverge without the restore
    w2.load_state(tmp_path / "s", restore_rng=True)
    _evolve(w2, 3)
    w2.spawn_cells([ms.random_genome(300) for _ in range(5)])
    assert list(w2.cell_genomes) == list(w.cell_genomes)
    assert list(w2.cell_labels) == list(w.cell_labels)
    assert torch.equal(w2.cell_positions, w.cell_positions)
    assert torch.equal(w2.cell_molecules, w.cell_molecules)
    assert torch.equal(w2.molecule_map, w.molecule_map)


class _RefClass:
    """Marks a stand-in class as the reference class ``_ref_path`` when pickled."""


def _ref_cls(path, base=object, **attrs):
    return type(path[1], (base,), {"_ref_path": path, **attrs})


def _reference_pickle(w) -> bytes:
    """A pickle with the reference's structure (magicsoup.world.World with list genomes, dense
    parameter tensors, Conv2d diffusion kernels; world.py:161-204, kinetics.py:390-460), built from
    a world of this package: the reference's own pickles cannot be produced here."""
    import io
    import pickle

    class RefPickler(pickle._Pickler):
        def save_global(self, obj, name=None):
            ref = obj.__dict__.get("_ref_path") if isinstance(obj, type) else None
            if ref is None:
                return super().save_global(obj, name)
            self.save(ref[0])
            self.save(ref[1])
            self.write(pickle.STACK_GLOBAL)
            self.memoize(obj)

    RW = _ref_cls(("magicsoup.world", "World"))
    RK = _ref_cls(("magicsoup.kinetics", "Kinetics"))
    RG = _ref_cls(("magicsoup.genetics", "Genetics"))
    maps = {}
    kin = w.kinetics
    for attr, cls_name in (("km_map", "_LogNormWeightMapFact"), ("vmax_map", "_LogNormWeightMapFact"),
                           ("sign_map", "_SignMapFact"), ("hill_map", "_HillMapFact"),
                           ("reaction_map", "_ReactionMapFact"), ("transport_map", "_TransporterMapFact"),
                           ("effector_map", "_RegulatoryMapFact")):
        o = _ref_cls(("magicsoup.kinetics", cls_name))()
        o.__dict__.update({k: v for k, v in vars(getattr(kin, attr)).items() if isinstance(v, torch.Tensor)})
        maps[attr] = o
    rk = RK()
    rk.__dict__.update(abs_temp=kin.abs_temp, device="cpu", mol_names=list(kin.mol_names),
                       mol_energies=kin.mol_energies.clone(), **{k: getattr(kin, k).clone() for k in
                                                                ("Ke", "Kmf", "Kmb", "Kmr", "Vmax", "N", "Nf", "Nb", "A")},
                       **maps, km_2_idxs=kin.km_2_idxs, vmax_2_idxs=kin.vmax_2_idxs, sign_2_idxs=kin.sign_2_idxs,
                       hill_2_idxs=kin.hill_2_idxs, trnsp_2_idxs=kin.trnsp_2_idxs, regul_2_idxs=kin.regul_2_idxs,
                       catal_2_idxs=kin.catal_2_idxs)
    rg = RG()
    g = w.genetics
    rg.__dict__.update({k: getattr(g, k) for k in ("start_codons", "stop_codons", "dom_size", "dom_type_size",
                                                   "domain_types", "domain_map", "one_codon_map", "two_codon_map",
                                                   "idx_2_one_codon", "idx_2_two_codon")})
    convs = []
    for a, b in w._diffusion:
        c = torch.nn.Conv2d(1, 1, 3, padding=1, padding_mode="circular", bias=False)
        c.weight.data = torch.tensor([[a, a, a], [a, b, a], [a, a, a]], dtype=torch.float32).view(1, 1, 3, 3)
        c.weight.requires_grad_(False)
        convs.append(c)
    rw = RW()
    rw.__dict__.update(device="cpu", batch_size=None, map_size=w.map_size, abs_temp=w.abs_temp, chemistry=w.chemistry,
                       genetics=rg, kinetics=rk, _mol_degrads=list(w._mol_degrads), _diffusion=convs,
                       _permeation=list(w._permeation), n_molecules=w.n_molecules,
                       _int_mol_idxs=list(w._int_mol_idxs), _ext_mol_idxs=list(w._ext_mol_idxs), n_cells=w.n_cells,
                       cell_genomes=list(w.cell_genomes), cell_labels=list(w.cell_labels), cell_map=w.cell_map.clone(),
                       cell_positions=w.cell_positions.clone(), cell_lifetimes=w.cell_lifetimes.clone(),
                       cell_divisions=w.cell_divisions.clone(), cell_molecules=w.cell_molecules.clone(),
                       molecule_map=w.molecule_map.clone())
    buf = io.BytesIO()
    RefPickler(buf, protocol=4).dump(rw)
    return buf.getvalue()


def test_from_file_reads_reference_layout_pickle(tmp_path):
    """World.from_file converts a reference-layout pickle (magicsoup.world.World etc.) into this
    package's World: same cells, maps, parameters and diffusion weights; usable afterwards.
    Parity unpinned: no reference pickle fixture exists, the file is built with the reference's
    structure (world.py:161-204)."""
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    ms.set_seed(3)
    w = ms.World(chemistry=CHEMISTRY, map_size=16)
    w.spawn_cells([ms.random_genome(500) for _ in range(30)])
    w.cell_lifetimes[3] = 7
    w._diffusion[0] = (0.05, 0.6)  # a non-default kernel must survive the round trip
    (tmp_path / "world.pkl").write_bytes(_reference_pickle(w))
    w2 = ms.World.from_file(tmp_path)
    assert type(w2) is ms.World and w2.n_cells == w.n_cells
    assert list(w2.cell_genomes) == list(w.cell_genomes)
    assert list(w2.cell_labels) == list(w.cell_labels)
    for k in ("cell_positions", "cell_lifetimes", "cell_divisions", "cell_molecules", "molecule_map", "cell_map"):
        assert torch.equal(getattr(w2, k), getattr(w, k)), k
    for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke"):
        assert torch.equal(getattr(w2.kinetics, k), getattr(w.kinetics, k)), k
    got = [x for ab in w2._diffusion for x in ab]
    want = [x for ab in w._diffusion for x in ab]
    assert got == pytest.approx(want, rel=1e-6)  # (fp32 kernel weights)
    assert w2.genetics.two_codon_map == w.genetics.two_codon_map
    w.enzymatic_activity()
    w2.enzymatic_activity()
    assert torch.equal(w2.cell_molecules, w.cell_molecules)
    w2.spawn_cells([ms.random_genome(300)])  # the converted world keeps working
    w2.diffuse_molecules()


def test_world_unpickler_refuses_foreign_globals(tmp_path):
    """from_file runs nothing a pickle names outside magicsoup / torch tensor rebuilds."""
    import os
    import pickle

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    (tmp_path / "world.pkl").write_bytes(pickle.dumps(Evil()))
    with pytest.raises(pickle.UnpicklingError):
        ms.World.from_file(tmp_path)


@pytest.mark.parametrize("payload", [
    # protocol 0 INST: World(...) -- a constructor that would allocate a map
    b"(I64\ni" b"magicsoup_amd.models.world\nWorld\n.",
    # OBJ: the class and its args after a MARK
    b"(cmagicsoup_amd.models.world\nWorld\nI64\no.",
    # NEWOBJ on a torch storage class (``__new__`` allocates what the file asks for)
    b"\x80\x02ctorch\nFloatStorage\nJ\x00\x00\x00\x40\x85\x81.",
])
def test_world_unpickler_refuses_constructor_opcodes(tmp_path, payload):
    """INST / OBJ may not call a data class (only REDUCE-callable containers); NEWOBJ may not create
    torch storages."""
    import pickle

    (tmp_path / "world.pkl").write_bytes(payload)
    with pytest.raises(pickle.UnpicklingError):
        ms.World.from_file(tmp_path)


def test_kill_divide_matches_kill_then_divide():
    """World.kill_divide_t(kill, divide) == kill_cells(kill) + divide_cells_t(divide[~kill]) (the
    bench loop's fused call), and ``last_kill`` records the counts."""
    import copy

    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    ms.set_seed(5)
    torch.manual_seed(5)
    base = ms.World(chemistry=CHEMISTRY, map_size=24)
    base.spawn_cells([ms.random_genome(300) for _ in range(150)])
    base.enzymatic_activity()
    atp = CHEMISTRY.molname_2_idx["ATP"]
    a = base.cell_molecules[:, atp]
    kill = a < torch.quantile(a, 0.3)
    div = (a > torch.quantile(a, 0.5)) & ~kill
    w1, w2 = copy.deepcopy(base), copy.deepcopy(base)
    ms.set_seed(9)
    w1.kill_divide_t(kill, div)
    ms.set_seed(9)
    n = w2.n_cells
    w2.kill_cells(kill)
    after = w2.n_cells
    w2.divide_cells_t(div[~kill])
    assert w1.last_kill == (n, after)
    assert w1.n_cells == w2.n_cells > after
    for k in ("cell_molecules", "cell_positions", "cell_lifetimes", "cell_divisions", "molecule_map", "cell_map"):
        assert torch.equal(getattr(w1, k), getattr(w2, k)), k
    assert list(w1.cell_genomes) == list(w2.cell_genomes)
    w1.check_invariants()
    with pytest.raises(ValueError):
        w1.kill_divide_t(kill, div)  # masks of the old population


def test_reserve_cells_keeps_state_and_results():
    """World.reserve_cells pre-allocates capacity; the world then evolves exactly as without it."""
    import copy

    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    ms.set_seed(6)
    w = ms.World(chemistry=CHEMISTRY, map_size=32)
    w.spawn_cells([ms.random_genome(300) for _ in range(40)])
    w2 = copy.deepcopy(w)
    w2.reserve_cells(500, genome_len=330)
    assert w2._cols["cell_molecules"].buf.size(0) >= 500
    for x in (w, w2):
        ms.set_seed(7)
        x.spawn_cells([ms.random_genome(300) for _ in range(60)])
        x.enzymatic_activity()
    assert torch.equal(w.cell_molecules, w2.cell_molecules)
    assert torch.equal(w.kinetics.Vmax, w2.kinetics.Vmax)
    w2.check_invariants()


def test_kill_divide_where_matches_masks():
    """kill_divide_where(molecule, below, above, cost) == the reference loop's masks + kill_divide_t."""
    import copy

    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    ms.set_seed(8)
    base = ms.World(chemistry=CHEMISTRY, map_size=24)
    base.spawn_cells([ms.random_genome(300) for _ in range(150)])
    base.enzymatic_activity()
    atp = CHEMISTRY.molname_2_idx["ATP"]
    a = base.cell_molecules[:, atp]
    lo, hi = float(torch.quantile(a, 0.3)), float(torch.quantile(a, 0.6))
    w1, w2 = copy.deepcopy(base), copy.deepcopy(base)
    ms.set_seed(2)
    w1.kill_divide_where("ATP", lo, hi, 0.5)
    ms.set_seed(2)
    b = w2.cell_molecules[:, atp]
    kill = b < lo
    div = (b > hi) & ~kill
    b -= 0.5 * div
    w2.kill_divide_t(kill, div)
    for k in ("cell_molecules", "cell_positions", "cell_divisions", "molecule_map", "cell_map"):
        assert torch.equal(getattr(w1, k), getattr(w2, k)), k
    assert w1.last_kill == w2.last_kill
    n = w1.n_cells
    w1.kill_divide_where(atp, -1.0, 1e9, kill_fraction=0.5)  # dilution only: about half die
    assert 0.25 * n < w1.n_cells < 0.75 * n
