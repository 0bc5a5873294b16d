"""DistributedWorld on the GPU: 2 ranks sharing one MI355X (gloo, host-staged exchanges), so the
strip-geometry HIP kernels (halo rows, no x wrap, claims into halo rows) run for real. The RCCL
transport itself is exercised by the multi-GPU bench."""
import copy

import pytest
import torch

from tests.dist_utils import run_ranks

pytestmark = pytest.mark.gpu


def _chem():
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    return CHEMISTRY


def _body_physics(rank, ws):
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    def world():
        ms.set_seed(3)
        torch.manual_seed(3)
        w = ms.World(chemistry=_chem(), map_size=64, seed=3, device="cpu")
        w.spawn_cells(gen_genomes(600, 300))
        return w

    # built on the CPU (deterministic placement) so both ranks scatter the same global world
    g = world()
    ref = copy.deepcopy(g).to("cuda")
    dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=5, device="cuda")
    dw.scatter_from(g)
    for _ in range(3):
        for w in (ref, dw):
            w.diffuse_molecules()
            w.enzymatic_activity()
            w.degrade_molecules()
    full = dw.gather()
    if rank == 0:
        assert torch.allclose(full.molecule_map, ref.molecule_map.cpu(), rtol=1e-4, atol=1e-4)
        ka = full.cell_positions.long() @ torch.tensor([64, 1])
        kb = ref.cell_positions.long().cpu() @ torch.tensor([64, 1])
        oa, ob = torch.argsort(ka), torch.argsort(kb)
        close = torch.isclose(full.cell_molecules[oa], ref.cell_molecules.cpu()[ob], rtol=1e-3, atol=1e-3)
        assert close.all(dim=1).float().mean() > 0.99


def test_gpu_distributed_physics_match_single_process():
    run_ranks(_body_physics, 2, timeout=600)


def _by_position(w, C):
    key = w.cell_positions.long().cpu() @ torch.tensor([C, 1])
    return torch.argsort(key)


def _body_physics_stepwise(rank, ws):
    """Per-op exactness against a single-process world that restarts from the gathered distributed
    state before every op (no drift between the two): the activity -- whose early exits are global
    decisions, the all-reduced flags here and the population-wide `any` there -- gives every cell the
    same bits; degradation too; diffusion + permeation agree to float rounding (the mass correction
    sums its global totals in another order)."""
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    C = 64
    ms.set_seed(4)
    torch.manual_seed(4)
    g = ms.World(chemistry=_chem(), map_size=C, seed=4, device="cpu")
    g.spawn_cells(gen_genomes(700, 300))
    dw = DistributedWorld(chemistry=_chem(), map_size=C, seed=6, device="cuda")
    dw.scatter_from(g)
    checked = {"activity": 0, "degrade": 0, "diffuse": 0}
    for it in range(3):
        for op in ("enzymatic_activity", "degrade_molecules", "diffuse_molecules"):
            ref = dw.gather()
            if rank == 0:
                ref = ref.to("cuda")
                getattr(ref, op)()
            getattr(dw, op)()
            full = dw.gather()
            if rank != 0:
                continue
            ref = ref.to("cpu")
            oa, ob = _by_position(full, C), _by_position(ref, C)
            assert torch.equal(full.cell_positions[oa], ref.cell_positions[ob])
            if op == "diffuse_molecules":
                assert torch.allclose(full.molecule_map, ref.molecule_map, rtol=2e-6, atol=1e-6)
                assert torch.allclose(full.cell_molecules[oa], ref.cell_molecules[ob], rtol=2e-6, atol=1e-6)
                checked["diffuse"] += 1
            else:
                a, b = full.cell_molecules[oa], ref.cell_molecules[ob]
                bad = (a != b).any(dim=1)
                assert not bad.any(), (op, it, int(bad.sum()), float((a - b).abs().max()),
                                       float(((a - b).abs() / b.abs().clamp(min=1e-30)).max()))
                assert torch.equal(full.molecule_map, ref.molecule_map), (op, it)
                checked["activity" if op == "enzymatic_activity" else "degrade"] += 1
    if rank == 0:
        assert checked == {"activity": 3, "degrade": 3, "diffuse": 3}


def test_gpu_distributed_physics_exact_per_op():
    run_ranks(_body_physics_stepwise, 2, timeout=600)


def _body_uniform_reposition_gpu(rank, ws):
    """reposition_cells(uniform=True) on GPU strips: some cells change rank, none is lost or
    duplicated, each keeps its molecules, occupancy stays consistent."""
    import torch.distributed as dist

    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(8)
    torch.manual_seed(8)
    g = ms.World(chemistry=_chem(), map_size=64, seed=8, device="cpu")
    g.spawn_cells(gen_genomes(900, 300))
    dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=9, device="cuda")
    dw.scatter_from(g)
    before = dw.gather()
    for _ in range(2):
        dw.reposition_cells(None, uniform=True)
        pos = dw.cell_positions.long()
        assert bool(((pos[:, 0] >= 1) & (pos[:, 0] <= dw.H)).all())
        assert int(dw.owned_cell_map().sum()) == dw.n_cells
    t = torch.tensor([dw.migrated["moved_out"]])
    dist.all_reduce(t)
    full = dw.gather()
    if rank == 0:
        assert full.n_cells == before.n_cells and int(full.cell_map.sum()) == full.n_cells
        key = lambda w: sorted(zip(w.cell_genomes, [tuple(r) for r in w.cell_molecules.tolist()]))
        assert key(full) == key(before)
        assert int(t) > 0


def test_gpu_distributed_uniform_reposition():
    run_ranks(_body_uniform_reposition_gpu, 2, timeout=600)


def _body_steps(rank, ws):
    import torch.distributed as dist

    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    dw = DistributedWorld(chemistry=_chem(), map_size=128, seed=9, device="cuda")
    dw.spawn_cells(gen_genomes(2000, 300))
    atp = _chem().molname_2_idx["ATP"]
    tot0 = dw.owned_molecule_map().double().sum(dim=[1, 2]) + dw.cell_molecules.double().sum(0)
    dist.all_reduce(tot0)
    for it in range(4):
        dw.enzymatic_activity()
        dw.kill_cells(torch.nonzero(dw.cell_molecules[:, atp] < 1.0).flatten())
        repl = dw.cell_molecules[:, atp] > 5.0
        dw.cell_molecules[:, atp] -= 4.0 * repl
        # index list and boolean mask (placement over the mask, no compaction first)
        dw.divide_cells_t(torch.nonzero(repl).flatten() if it % 2 else repl)
        dw.recombinate_cells(p=1e-4)
        dw.mutate_cells(p=1e-4)
        dw.degrade_molecules()
        dw.diffuse_molecules()
        dw.move_cells()
        dw.increment_cell_lifetimes()
        pos = dw.cell_positions.long()
        assert bool(((pos[:, 0] >= 1) & (pos[:, 0] <= dw.H)).all())
        assert int(dw.owned_cell_map().sum()) == dw.n_cells
        assert bool(dw.cell_map[pos[:, 0], pos[:, 1]].all())
        assert torch.isfinite(dw.molecule_map).all()
    # division / movement conserve molecules across ranks
    tot = dw.owned_molecule_map().double().sum(dim=[1, 2]) + dw.cell_molecules.double().sum(0)
    dist.all_reduce(tot)
    assert torch.isfinite(tot).all()
    full = dw.gather()
    if rank == 0:
        n = full.n_cells
        p = full.cell_positions.long()
        assert (p[:, 0] * 128 + p[:, 1]).unique().numel() == n
        assert int(full.cell_map.sum()) == n


def test_gpu_distributed_steps_keep_invariants():
    run_ranks(_body_steps, 2, timeout=600)


def _body_rccl_self(rank, ws):
    """The native RCCL communicator on one GPU rank: exchanges with itself (up == down == self on a
    one-rank ring) and all-reduces, enqueued on the current stream between kernels."""
    from magicsoup_amd.parallel.comm import RcclComm, make_comm

    comm = make_comm(None, 0, 1, "cuda")
    assert isinstance(comm, RcclComm) and comm.up == comm.down == 0
    a = torch.arange(1000, dtype=torch.float32, device="cuda")
    b = torch.arange(1000, 1500, dtype=torch.int32, device="cuda")
    ra = torch.empty_like(a)
    rb = torch.empty_like(b)
    # to_up arrives as from_down, to_down as from_up (both at ourselves)
    comm.exchange(a, b, ra, rb)
    torch.cuda.synchronize()
    assert torch.equal(ra, a) and torch.equal(rb, b)
    t = torch.tensor([3.0, -1.0], dtype=torch.float64, device="cuda")
    comm.allreduce_(t, "max")
    f = torch.tensor([1, 0, 2, 0], dtype=torch.int32, device="cuda")
    comm.allreduce_(f, "sum")
    torch.cuda.synchronize()
    assert t.tolist() == [3.0, -1.0] and f.tolist() == [1, 0, 2, 0]
    comm.check()
    comm.close()


def test_native_rccl_comm_single_rank():
    run_ranks(_body_rccl_self, 1, timeout=300, backend="nccl")


@pytest.mark.parametrize("p", [0.01, 5e-4])  # synchronous path (high rate) / device genome pipeline
def test_gpu_boundary_recombination_is_symmetric(p):
    from tests.test_distributed import _body_boundary_pairs

    run_ranks(_body_boundary_pairs, 2, "cuda", p, 0.25 if p > 1e-3 else 0.0, timeout=300)


def _body_spec_fallback(rank, ws):
    """The decomposed speculative integration: one all-reduce of the speculative flags decides for
    the whole job. Voiding the speculation on rank 0 only (integrate mode bit 9) must make BOTH ranks
    run the exact per-part launches, and those give the same state bit for bit as the speculation
    that held."""
    import magicsoup_amd as ms
    from magicsoup_amd.ops import hip_ops, native
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(4)
    torch.manual_seed(4)
    g = ms.World(chemistry=_chem(), map_size=64, seed=4, device="cpu")
    g.spawn_cells(gen_genomes(800, 300))
    dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=5, device="cuda")
    dw.scatter_from(g)
    dw.diffuse_molecules()
    cm0, mm0 = dw.cell_molecules.clone(), dw.molecule_map.clone()
    spec = hip_ops._scratch(dw.kinetics).bufs

    dw.enzymatic_activity()
    torch.cuda.synchronize()
    held = spec["spec"][4:17].tolist()
    cm1, mm1 = dw.cell_molecules.clone(), dw.molecule_map.clone()
    assert held[12] == 0 and all(held[:12])  # the speculation held on the whole job

    dw.cell_molecules = cm0.clone()
    dw.molecule_map = mm0.clone()
    if rank == 0:
        native.hip().set_integrate_mode(512)
    try:
        dw.enzymatic_activity()
        torch.cuda.synchronize()
    finally:
        native.hip().set_integrate_mode(0)
    assert spec["spec"][16].item() == 1  # global: void on every rank
    assert torch.equal(dw.cell_molecules, cm1)
    assert torch.equal(dw.molecule_map, mm1)


def test_gpu_distributed_speculation_is_a_global_decision():
    run_ranks(_body_spec_fallback, 2, timeout=600)


def _body_halo_overlap(rank, ws):
    """One rank, strips over RCCL (virtual: the rank is its own neighbour): the stencil split into
    interior rows (issued while the halo rows are exchanged on a stream of their own) and the two
    boundary rows gives the single-launch result and the plain world's (up to the order of the fp64
    mass sums behind the correction)."""
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld

    dw = DistributedWorld(chemistry=_chem(), map_size=256, seed=2, device="cuda", strips=True)
    assert dw._halo_async
    mm0 = dw.molecule_map.clone()
    out = {}
    for split in (True, False):
        dw.molecule_map = mm0.clone()
        dw.__dict__["_halo_async"] = split
        for _ in range(3):
            dw.degrade_molecules()
            dw.diffuse_molecules()
        out[split] = dw.owned_molecule_map().clone()
    w = ms.World(chemistry=_chem(), map_size=256, seed=2, device="cuda")
    w.molecule_map = mm0[:, 1:257].clone()
    for _ in range(3):
        w.degrade_molecules()
        w.diffuse_molecules()
    torch.testing.assert_close(out[True], out[False], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(out[True], w.molecule_map, rtol=1e-6, atol=1e-6)


def test_gpu_halo_exchange_overlaps_interior_stencil():
    run_ranks(_body_halo_overlap, 1, timeout=300, backend="nccl")


def _body_native_dist_integrate(rank, ws):
    """One rank over RCCL (virtual strips): the decomposed integration runs natively with its flag
    all-reduces (kinetics.hip integrate_dist) and gives the plain world's result bit for bit."""
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(6)
    torch.manual_seed(6)
    w = ms.World(chemistry=_chem(), map_size=128, seed=6, device="cuda")
    w.spawn_cells(gen_genomes(1500, 300))
    dw = DistributedWorld(chemistry=_chem(), map_size=128, seed=7, device="cuda", strips=True)
    dw.adopt_maps(w)
    dw.scatter_from(w, maps=False)
    assert dw._rccl_handle() is not None
    calls = []
    hook = dw._allreduce_flags
    dw.__dict__["_allreduce_flags"] = lambda f: (calls.append(int(f.numel())), hook(f))
    for _ in range(2):
        w.enzymatic_activity()
        dw.enzymatic_activity()
    assert calls == []  # (the all-reduces were issued natively)
    assert torch.equal(dw.cell_molecules, w.cell_molecules)
    assert torch.equal(dw.owned_molecule_map(), w.molecule_map)


def test_gpu_native_decomposed_integration_matches_plain_world():
    run_ranks(_body_native_dist_integrate, 1, timeout=300, backend="nccl")


def _body_native_divide(rank, ws):
    """One rank over RCCL (virtual strips, the rank is its own neighbour): divide_cells over a mask
    as the two native calls (fast.hip fast_dist_divide_a / _b) gives the Python protocol's result
    exactly -- placements, migrated children, molecules, genomes, labels and parameters."""
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from magicsoup_amd.parallel import dist_world as dwm
    from tests.conftest import gen_genomes

    ms.set_seed(8)
    torch.manual_seed(8)
    w = ms.World(chemistry=_chem(), map_size=64, seed=8, device="cpu")
    w.spawn_cells(gen_genomes(1200, 300))
    atp = _chem().molname_2_idx["ATP"]
    out = {}
    for native in (True, False):
        dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=9, device="cuda", strips=True)
        dw.adopt_maps(w)
        dw.scatter_from(w, maps=False)
        dwm._NATIVE_DIVIDE = native
        try:
            for it in range(3):
                dw.enzymatic_activity()
                mask = dw.cell_molecules[:, atp] > 2.0
                ms.set_seed(11 + it)
                par, ch = dw.divide_cells_t(mask)
        finally:
            dwm._NATIVE_DIVIDE = True
        dw.enzymatic_activity()
        torch.cuda.synchronize()
        out[native] = (par.cpu(), ch.cpu(), dw.cell_positions.cpu(), dw.cell_molecules.cpu(), dw.cell_divisions.cpu(),
                       dw.cell_lifetimes.cpu(), list(dw.cell_genomes), list(dw.cell_labels), dw.cell_map.cpu(),
                       dict(dw.migrated))
        dw.close()
    a, b = out[True], out[False]
    assert a[9]["divided_in"] > 0  # children crossed the (self-)boundary
    for x, y in zip(a[:6], b[:6]):
        assert torch.equal(x, y)
    assert a[6] == b[6] and a[7] == b[7] and torch.equal(a[8], b[8]) and a[9] == b[9]


def test_gpu_native_strip_divide_matches_python_protocol():
    run_ranks(_body_native_divide, 1, timeout=300, backend="nccl")


def _body_native_xb(rank, ws):
    """One rank over RCCL (virtual strips): the collective part of the strip-boundary recombination
    as one native call (dist.hip xb_begin) gives the Python protocol's genomes exactly."""
    import random

    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from magicsoup_amd.parallel import dist_world as dwm
    from tests.conftest import gen_genomes

    ms.set_seed(12)
    torch.manual_seed(12)
    w = ms.World(chemistry=_chem(), map_size=64, seed=12, device="cpu")
    w.spawn_cells(gen_genomes(1500, 300))
    out = {}
    real = dwm.RcclComm
    for native in (True, False):
        random.seed(77)
        dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=13, device="cuda", strips=True)
        dw.adopt_maps(w)
        dw.scatter_from(w, maps=False)
        if not native:
            dwm.RcclComm = type("NotRccl", (), {})  # the isinstance check fails: the Python exchanges
        try:
            for it in range(3):
                ms.set_seed(40 + it)
                dw.recombinate_cells(p=2e-3)
            genomes = list(dw.cell_genomes)
        finally:
            dwm.RcclComm = real
        out[native] = (genomes, dw.kinetics.N.cpu().clone())
        dw.close()
    assert out[True][0] == out[False][0]
    assert torch.equal(out[True][1], out[False][1])
    assert out[True][0] != list(w.cell_genomes)  # something recombined


def test_gpu_native_boundary_recombination_matches_python_protocol():
    run_ranks(_body_native_xb, 1, timeout=300, backend="nccl")


def _body_lazy_strip_divide(rank, ws):
    """One rank over RCCL (virtual strips): the reference loop with divide_cells_t(mask, lazy=True)
    -- phase B deferred to the next diffusion, the boundary recombination issued at the flush --
    ends in exactly the state of the eager protocol (positions, molecules, divisions, lifetimes,
    genomes, labels, parameters, occupancy, map, migration counters)."""
    import random

    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(21)
    torch.manual_seed(21)
    w = ms.World(chemistry=_chem(), map_size=64, seed=21, device="cpu")
    w.spawn_cells(gen_genomes(1200, 300))
    atp = _chem().molname_2_idx["ATP"]
    out = {}
    rebuilds = {}
    orig_rebuild = DistributedWorld._rebuild_arrivals

    def counting_rebuild(self, arr):
        rebuilds[self._lazy_tag] = rebuilds.get(self._lazy_tag, 0) + 1
        return orig_rebuild(self, arr)

    DistributedWorld._rebuild_arrivals = counting_rebuild
    for lazy in (False, True, "again"):
        random.seed(5)
        dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=22, device="cuda", strips=True)
        dw.__dict__["_lazy_tag"] = lazy
        dw.adopt_maps(w)
        dw.scatter_from(w, maps=False)
        ms.set_seed(23)
        for it in range(4):
            dw.enzymatic_activity()
            dw.kill_cells(dw.cell_molecules[:, atp] < 0.5)
            repl = dw.cell_molecules[:, atp] > 2.0
            dw.cell_molecules[:, atp] -= 1.0 * repl
            r = dw.divide_cells_t(repl, lazy=lazy is True)
            assert (r is None) == (lazy is True)
            if lazy is True:
                assert dw.__dict__.get("_count_pending") is not None
            # (a rate whose worst-case pair count stays 8 sigma inside the merged chain's capacity:
            # genome_pipeline._pair_cap; above it a strip issues the recombination on its own)
            dw.recombinate_cells(p=2e-5)
            dw.mutate_cells(p=1e-4)
            dw.degrade_molecules()
            dw.diffuse_molecules()
            assert dw.__dict__.get("_count_pending") is None  # completed before the stencil
            dw.increment_cell_lifetimes()
        dw.synchronize()
        out[lazy] = (dw.cell_positions.cpu(), dw.cell_molecules.cpu(), dw.cell_divisions.cpu(),
                     dw.cell_lifetimes.cpu(), dw.cell_map.cpu(), dw.owned_molecule_map().cpu(), dw.kinetics.N.cpu().clone(),
                     list(dw.cell_genomes), list(dw.cell_labels), dict(dw.migrated))
        dw.close()
    names = ("positions", "molecules", "divisions", "lifetimes", "cell_map", "molecule_map", "N", "genomes",
             "labels", "migrated")

    def diff(a, b):
        bad = []
        for name, x, y in zip(names, a, b):
            same = torch.equal(x, y) if isinstance(x, torch.Tensor) and x.shape == y.shape else x == y
            if not same:
                extra = ""
                if isinstance(x, torch.Tensor) and x.shape == y.shape and x.is_floating_point():
                    extra = f" max abs diff {float((x - y).abs().max())}"
                elif isinstance(x, torch.Tensor):
                    extra = f" shapes {tuple(x.shape)} {tuple(y.shape)}"
                bad.append(name + extra)
        return bad

    DistributedWorld._rebuild_arrivals = orig_rebuild
    a, b, c = out[False], out[True], out["again"]
    assert a[9]["divided_in"] > 0
    # eager: the arrivals get a rebuild chain of their own; lazy: the queued genome chain builds them
    assert rebuilds.get(False, 0) > 0 and rebuilds.get(True, 0) == 0, rebuilds
    assert not diff(a, c), f"eager protocol not reproducible: {diff(a, c)}"
    assert not diff(a, b), f"lazy differs from eager: {diff(a, b)} ({a[9]} vs {b[9]})"


def test_gpu_lazy_strip_divide_matches_eager():
    run_ranks(_body_lazy_strip_divide, 1, timeout=300, backend="nccl")


def _body_lazy_divide_after_closed_comm(rank, ws):
    """A communicator that existed and was closed leaves the peer-failure guard registered but with
    no live communicator: a lazy division's count must still wait for the division's kernels
    (the guard returned without waiting and the count was read stale)."""
    import magicsoup_amd as ms
    from magicsoup_amd.ops import hip_ops
    from magicsoup_amd.parallel.comm import make_comm

    comm = make_comm(None, 0, 1, "cuda")
    comm.close()
    del comm
    assert hip_ops._GUARD  # registered once, stays registered
    chem = _chem()
    atp = chem.molname_2_idx["ATP"]
    ms.set_seed(11)
    torch.manual_seed(11)
    base = ms.World(chemistry=chem, map_size=96, device="cuda", seed=11)
    base.spawn_cells([ms.random_genome(400) for _ in range(2500)])
    base.synchronize()
    for lazy in (False, True):
        # (one spawned world copied: GPU spawn placement races, so two spawns differ)
        w = copy.deepcopy(base)
        ms.set_seed(12)
        w.enzymatic_activity()
        repl = w.cell_molecules[:, atp] > -1.0  # every cell tries to divide
        w.divide_cells_t(repl, lazy=lazy)
        n = w.n_cells
        w.check_invariants("lazy division after a closed communicator")
        if lazy:
            assert n == n_sync, (n, n_sync)
        else:
            n_sync = n
            assert n > 2500


def test_lazy_division_waits_after_communicator_closed():
    run_ranks(_body_lazy_divide_after_closed_comm, 1, timeout=300, backend="nccl")


def _body_dense_strip_recombination(rank, ws):
    """A dense strip at a recombination rate whose pair count can exceed the device chain's pair
    capacity: the merged recombinate + mutate chain must not be issued with the boundary results
    (a skip there cannot be replayed); the strip takes the synchronous path instead."""
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(31)
    torch.manual_seed(31)
    dw = DistributedWorld(chemistry=_chem(), map_size=48, seed=31, device="cuda", strips=True)
    dw.spawn_cells(gen_genomes(2100, 500))
    n0 = dw.n_cells
    for _ in range(3):
        dw.recombinate_cells(p=3e-4)
        dw.mutate_cells(p=1e-4)
        dw.diffuse_molecules()
        dw.synchronize()
    assert dw.n_cells == n0
    assert sum(len(g) for g in dw.cell_genomes) > 0
    dw.check_invariants("dense strip recombination")
    dw.close()


def test_dense_strip_recombination_does_not_skip_boundary_results():
    run_ranks(_body_dense_strip_recombination, 1, timeout=300, backend="nccl")


def _body_strip_kill_divide_where(rank, ws):
    """A strip world's kill_divide_where (native masks, kill, division mask compacted on the device,
    lazy strip division) evolves the strip exactly as the torch masks + kill_cells + divide_cells_t
    do."""
    import magicsoup_amd as ms
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(41)
    torch.manual_seed(41)
    w = ms.World(chemistry=_chem(), map_size=64, seed=41, device="cpu")
    w.spawn_cells(gen_genomes(1200, 300))
    atp = _chem().molname_2_idx["ATP"]
    from magicsoup_amd.parallel import dist_world

    out, kills = {}, {}
    lazy0, early0 = dist_world._LAZY_KILL, dist_world._EARLY_STENCIL
    # masks: torch masks + kill_cells + lazy divide; eager: native masks, the kill's read-back, lazy
    # divide; lazy: kill and phase A in one call, the survivor count read with phase A's counts
    # (*_f: with a chemostat dilution, whose draws the torch masks cannot reproduce)
    # (late: the stencil after phase B on the compute stream; the others issue phase B after the
    # stencil on the side stream, DistributedWorld._diffuse_early)
    for fused in ("masks", "eager", "lazy", "late", "eager_f", "lazy_f"):
        dist_world._LAZY_KILL = fused.startswith("lazy") or fused == "late"
        dist_world._EARLY_STENCIL = fused != "late"
        dw = DistributedWorld(chemistry=_chem(), map_size=64, seed=42, device="cuda", strips=True)
        dw.adopt_maps(w)
        dw.scatter_from(w, maps=False)
        ms.set_seed(43)
        for it in range(3):
            dw.enzymatic_activity()
            if fused != "masks":
                dw.kill_divide_where(atp, 0.5, 2.0, 1.0, kill_fraction=0.2 if fused.endswith("_f") else 0.0)
            else:
                a = dw.cell_molecules[:, atp]
                kill = a < 0.5
                repl = (a > 2.0) & ~kill
                a -= 1.0 * repl
                dw.kill_cells(kill)
                dw.divide_cells_t(repl[~kill], lazy=True)
            dw.degrade_molecules()
            dw.diffuse_molecules()
            dw.increment_cell_lifetimes()
            if fused != "masks":  # (the diffusion completed the lazy division: the counts are in)
                kills.setdefault(fused, []).append(tuple(dw.last_kill))
        dw.synchronize()
        dw.check_invariants("strip kill_divide_where")
        out[fused] = (dw.cell_positions.cpu(), dw.cell_molecules.cpu(), dw.cell_divisions.cpu(), list(dw.cell_genomes))
        dw.close()
    dist_world._LAZY_KILL, dist_world._EARLY_STENCIL = lazy0, early0
    a = out["masks"]
    for k in ("eager", "lazy", "late"):
        b = out[k]
        assert all(torch.equal(x, y) for x, y in zip(a[:3], b[:3])) and a[3] == b[3], k
    assert kills["eager"] == kills["lazy"] == kills["late"] and kills["eager_f"] == kills["lazy_f"]
    a, b = out["eager_f"], out["lazy_f"]
    assert all(torch.equal(x, y) for x, y in zip(a[:3], b[:3])) and a[3] == b[3]
    assert kills["lazy_f"][0][1] < kills["lazy"][0][1]  # (the dilution killed cells)


def test_strip_kill_divide_where_matches_masks():
    run_ranks(_body_strip_kill_divide_where, 1, timeout=300, backend="nccl")


def test_gpu_sharded_state_matches_gathered(tmp_path):
    """The sharded checkpoint of GPU strips (2 gloo ranks sharing the device): shards written from
    device memory, the assembled reference layout byte-equal to the gathered save, shard and
    reference-file loads bit-exact, load -> save reproducing the files, exact resume."""
    from tests.test_distributed import _body_sharded_state

    run_ranks(_body_sharded_state, 2, str(tmp_path), "cuda", timeout=600)


def test_gpu_sharded_state_virtual_strip_over_rccl(tmp_path):
    """The same on one rank as a virtual strip over the native RCCL communicator."""
    from tests.test_distributed import _body_sharded_state

    run_ranks(_body_sharded_state, 1, str(tmp_path), "cuda", {"strips": True}, timeout=300, backend="nccl")
