"""Numerics of the gfx950 kernels against fp32 PyTorch / host references (GPU only)."""
import copy

import pytest
import torch

import magicsoup_amd as ms
from magicsoup_amd.models.kinetics import Kinetics
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY
from magicsoup_amd.ops import native
from tests.conftest import gen_genomes

pytestmark = pytest.mark.gpu


def _world(device, map_size=64, n=300, s=500, seed=1):
    ms.set_seed(seed)
    torch.manual_seed(seed)
    w = ms.World(chemistry=CHEMISTRY, map_size=map_size, device=device, seed=seed)
    if n:
        w.spawn_cells(gen_genomes(n, s))
    return w


def test_extension_is_gfx950():
    assert native.hip().device_arch().startswith("gfx950")


def test_translation_matches_host():
    genetics = ms.Genetics()
    # short genomes use LDS slots, the long ones (> 2048 nt) the global-slot pass
    genomes = gen_genomes(500, 800) + ["", "ATG", ms.random_genome(30), ms.random_genome(3000), ms.random_genome(9000)]
    genomes += gen_genomes(50, 1100) + gen_genomes(20, 2000)
    from magicsoup_amd.models.strings import pack_strings

    arr, lens = pack_strings(genomes)
    tok_h, np_h = genetics.tables.translate_tokens(arr, lens)
    from magicsoup_amd.models.strings import PoolArena
    from magicsoup_amd.ops import hip_ops

    pool = PoolArena("cuda")  # (the GPU genome store: ragged, one byte per nt)
    pool.append_packed(torch.from_numpy(arr), torch.from_numpy(lens))
    rows = torch.arange(len(genomes), device="cuda")
    tok_d, np_d = hip_ops.translate(genetics, pool, rows)
    assert torch.equal(np_d.cpu(), torch.as_tensor(np_h))
    assert torch.equal(tok_d.cpu(), torch.as_tensor(tok_h))


def test_translation_past_64k_nt_matches_host():
    """Genomes past 65535 nt (long evolving runs grow them by recombination) translate through the
    32-bit position layout of the global-slot pass (genetics.hip PosT<true>) with the host's tokens."""
    genetics = ms.Genetics()
    ms.set_seed(6)
    genomes = [ms.random_genome(70000), ms.random_genome(131072 + 5)] + gen_genomes(40, 600) + [ms.random_genome(5000)]
    # (long CDS lists -- more than kRankMax per strand -- take the sorted emission order)
    genomes += [ms.random_genome(n) for n in (4000, 8000, 16000, 30000, 12345)]
    from magicsoup_amd.models.strings import PoolArena, pack_strings
    from magicsoup_amd.ops import hip_ops

    arr, lens = pack_strings(genomes)
    tok_h, np_h = genetics.tables.translate_tokens(arr, lens)
    pool = PoolArena("cuda")
    pool.append_packed(torch.from_numpy(arr), torch.from_numpy(lens))
    rows = torch.arange(len(genomes), device="cuda")
    tok_d, np_d = hip_ops.translate(genetics, pool, rows)
    assert int(np_d[1]) > 1000  # (the 131k-nt genome's proteome)
    assert torch.equal(np_d.cpu(), torch.as_tensor(np_h))
    assert torch.equal(tok_d.cpu(), torch.as_tensor(tok_h))


def _copy_world_cpu_to_gpu(wc):
    wg = copy.deepcopy(wc)
    return wg.to("cuda")


@pytest.mark.parametrize("n", [200, 30000])
def test_param_build_matches_host(n):
    wc = _world("cpu", n=n, map_size=64 if n < 3000 else 256)
    rows = torch.arange(wc.n_cells)
    from magicsoup_amd.ops import world_ops, hip_ops, kinetics_ops

    tokens, nprot = world_ops.translate(wc, rows)
    wg = _copy_world_cpu_to_gpu(wc)
    kg = wg.kinetics
    for name in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke"):
        getattr(kg, name).zero_()
    full = nprot > 0
    kinetics_ops.build_params(kg, rows[full].int(), tokens[full].cuda())
    kc = wc.kinetics
    for name in ("N", "Nf", "Nb", "A"):
        assert torch.equal(getattr(kg, name).cpu()[full], getattr(kc, name)[full]), name
    for name in ("Kmr", "Kmf", "Kmb", "Vmax", "Ke"):
        a, b = getattr(kg, name).cpu()[full], getattr(kc, name)[full]
        # bit for bit: the Kmr powers are integer products in both builds (device powf differs from
        # the host's in the last bit, and a decomposed world's ranks build on the device what a
        # gathered world rebuilds on the host)
        assert torch.equal(a.nan_to_num(-7.0), b.nan_to_num(-7.0)), name


@pytest.mark.parametrize("n_iters", [0, 4])
def test_integrator_matches_torch_oracle(n_iters):
    w = _world("cuda", n=400)
    kin = w.kinetics
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()

    from magicsoup_amd.ops import kinetics_ops

    # torch oracle (stage-by-stage reference semantics)
    Xr = X.clone()
    for trim in (0.7, 0.2, 0.1):
        V = kin._get_velocities(X=Xr, Vmax=(kin.Vmax * trim).clamp(0.0))
        NV = kin.N.float() * V.unsqueeze(2)
        NVa = kin._get_negative_adjusted_nv(NV=NV, X=Xr)
        X1 = (Xr + NVa.sum(1)).clamp(min=0.0)
        Xr = kin._get_equilibrium_adjusted_x(X0=Xr, X1=X1, NV=NVa, V=V) if n_iters else X1
    Xk = X.clone()
    kinetics_ops.integrate(kin, Xk, trims=(0.7, 0.2, 0.1), n_iters=n_iters)
    assert torch.isfinite(Xk).all()
    assert (Xk >= 0).all()
    # The damping iterations branch on Q/Ke vs 1.5 / 0.67. When the negative-concentration guard
    # exhausts a species, X1 lands on +-1 ulp of 0 depending on the summation order (torch's
    # reduction tree vs our per-signal loop), and Q = 0 vs Q = tiny can flip such a decision. This is
    # a property of the reference algorithm (its CPU and CUDA paths differ the same way), so the
    # oracle comparison is per cell; exact agreement is required between our two native cores.
    close = torch.isclose(Xk, Xr, rtol=1e-3, atol=1e-3).all(dim=1).cpu().numpy()
    if n_iters == 0:
        assert close.mean() > 0.999, close.mean()
        return
    # decision-aware: only cells with a damping decision at a Q/Ke threshold (float64 population
    # oracle, relative margin 1e-3) may differ between two float32 operation orders
    import numpy as np

    from tests.test_kinetics import _oracle_population

    params = [{k: getattr(kin, k)[c].double().cpu().numpy() for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb",
                                                                       "Vmax", "Ke")} for c in range(X.size(0))]
    _, border = _oracle_population(params, X.double().cpu().numpy(), (0.7, 0.2, 0.1), n_iters, margin=1e-3)
    border = np.array(border)
    # (a cell counts as ill-conditioned when any of its decisions is: the bulk still agrees outright)
    assert close.mean() >= 0.9 and close[~border].all(), (close.mean(), np.nonzero(~close & ~border))


def test_integrator_matches_host_core():
    wc = _world("cpu", n=300)
    wg = _copy_world_cpu_to_gpu(wc)
    pos = wc.cell_positions.long()
    X = torch.cat([wc.cell_molecules, wc.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    Xc = wc.kinetics.integrate_signals(X)
    Xg = wg.kinetics.integrate_signals(X.cuda()).cpu()
    # same algorithm and operation order, no FMA contraction on either side; the device's exp / pow
    # may differ from the host libm by an ulp, which can only matter where a damping decision sits
    # on its Q/Ke threshold. Decision-aware: every cell whose decisions all clear the thresholds by
    # a relative margin of 1e-4 (float64 population oracle) must agree to 1e-5; no blanket allowance.
    import numpy as np

    from tests.test_kinetics import _oracle_population

    close = torch.isclose(Xg, Xc, rtol=1e-5, atol=1e-6).all(dim=1).numpy()
    kin = wc.kinetics
    params = [{k: getattr(kin, k)[c].double().numpy() for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax",
                                                               "Ke")} for c in range(X.size(0))]
    _, border = _oracle_population(params, X.double().numpy(), (0.7, 0.2, 0.1), 4, margin=1e-4)
    border = np.array(border)
    assert close[~border].all(), np.nonzero(~close & ~border)
    assert wg.kinetics.last_masks == wc.kinetics.last_masks


def test_huge_proteome_integrates_through_device_memory_slots():
    """A cell whose proteome overflows an LDS slot (1169 proteins here: 206 KiB of slot; long evolving
    runs grow such genomes by recombination) integrates through slots in device memory
    (kinetics.hip lds_slots) instead of failing, with the host core's results."""
    ms.set_seed(2)
    torch.manual_seed(2)
    wc = ms.World(chemistry=CHEMISTRY, map_size=32, device="cpu", seed=2)
    wc.spawn_cells([ms.random_genome(60000) for _ in range(3)] + gen_genomes(60, 500))
    assert wc.kinetics.N.size(1) > 1000
    wg = _copy_world_cpu_to_gpu(wc)
    for _ in range(2):
        wc.enzymatic_activity()
        wg.enzymatic_activity()
    assert torch.allclose(wg.cell_molecules.cpu(), wc.cell_molecules, rtol=1e-4, atol=1e-4)
    assert torch.allclose(wg.molecule_map.cpu(), wc.molecule_map, rtol=1e-4, atol=1e-4)


def test_proteome_past_8191_proteins_matches_host():
    """A proteome past the old 14-bit record count (a seeded 3000-step flagship run grew one of ~9600
    proteins): the record slot's 16-bit count names it (params.h), and its activity through
    device-memory integrator slots matches the host core."""
    from magicsoup_amd.models.kinetics import _REC_CNT_MASK, _REC_OFF_BITS

    ms.set_seed(5)
    torch.manual_seed(5)
    wc = ms.World(chemistry=CHEMISTRY, map_size=32, device="cpu", seed=5)
    wc.spawn_cells([ms.random_genome(460000)] + gen_genomes(30, 500))
    assert wc.kinetics.N.size(1) > 8191
    wg = _copy_world_cpu_to_gpu(wc)
    wg.kinetics._enter_slot_mode()  # (the copied dense rows become records)
    slot = wg.kinetics.__dict__["_slot"]
    cnt = (slot >> _REC_OFF_BITS) & _REC_CNT_MASK
    assert int(cnt.max()) > 8191
    wc.enzymatic_activity()
    wg.enzymatic_activity()
    assert torch.allclose(wg.cell_molecules.cpu(), wc.cell_molecules, rtol=1e-4, atol=1e-4)
    assert torch.allclose(wg.molecule_map.cpu(), wc.molecule_map, rtol=1e-4, atol=1e-4)
    # (a rebuild on the device path: every cell takes records of its own proteome's size, the giant
    # one past 8191; the copied dense rows were P records each)
    from magicsoup_amd.ops import world_ops

    wg._update_params_rows(torch.arange(wg.n_cells, device="cuda"))
    cnt2 = (wg.kinetics.__dict__["_slot"] >> _REC_OFF_BITS) & _REC_CNT_MASK
    _, nprot = world_ops.translate(wc, torch.arange(wc.n_cells))
    assert int(nprot[0]) > 8191
    assert torch.equal(cnt2.cpu(), nprot.to(torch.int64).cpu())
    wg.enzymatic_activity()
    wc.enzymatic_activity()
    assert torch.allclose(wg.cell_molecules.cpu(), wc.cell_molecules, rtol=1e-4, atol=1e-4)


def test_enzymatic_activity_matches_host():
    wc = _world("cpu", n=300)
    wg = _copy_world_cpu_to_gpu(wc)
    wc.enzymatic_activity()
    wg.enzymatic_activity()
    assert torch.allclose(wg.cell_molecules.cpu(), wc.cell_molecules, rtol=1e-4, atol=1e-4)
    assert torch.allclose(wg.molecule_map.cpu(), wc.molecule_map, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("size", [5, 33, 67, 256, 300, 1000])
def test_diffusion_matches_host(size):
    wc = _world("cpu", map_size=size, n=0)
    wg = _copy_world_cpu_to_gpu(wc)
    wc.degrade_molecules()
    wc.diffuse_molecules()
    wg.degrade_molecules()
    wg.diffuse_molecules()
    assert torch.allclose(wg.molecule_map.cpu(), wc.molecule_map, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("band", [16, 48, 64, 128])
@pytest.mark.parametrize("vec", [4, 8])
def test_diffusion_band_heights_match_host(band, vec):
    """The vector stencils' wave bands (set_stencil_band: taller bands re-read fewer halo rows) and
    both column widths give the host result for any band height, including bands taller than the
    map and partial last bands."""
    try:
        native.hip().set_stencil_band(band)
        native.hip().set_stencil_vec(vec)
        for size in (40, 200):
            wc = _world("cpu", map_size=size, n=0)
            wg = _copy_world_cpu_to_gpu(wc)
            for w in (wc, wg):
                w.degrade_molecules()
                w.diffuse_molecules()
            assert torch.allclose(wg.molecule_map.cpu(), wc.molecule_map, rtol=1e-5, atol=1e-5), size
    finally:
        native.hip().set_stencil_band(0)
        native.hip().set_stencil_vec(0)


def test_diffusion_conserves_mass():
    w = _world("cuda", map_size=512, n=0)
    before = w.molecule_map.double().sum(dim=[1, 2])
    for _ in range(10):
        w.diffuse_molecules()
    after = w.molecule_map.double().sum(dim=[1, 2])
    assert torch.all((after - before).abs() / before < 1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_reduced_precision_maps_track_fp32(dtype):
    """bf16/fp16 map storage: the kernels compute in fp32 and round once per store."""
    ref = _world("cuda", map_size=200, n=300)
    low = copy.deepcopy(ref)
    low.__dict__["map_dtype"] = dtype
    low.molecule_map = ref.molecule_map
    ref.molecule_map = low.molecule_map.float()  # start both from the same representable values
    assert low.molecule_map.dtype == dtype
    for w in (ref, low):
        for _ in range(3):
            w.enzymatic_activity()
            w.degrade_molecules()
            w.diffuse_molecules()
    eps = 2.0**-7 if dtype == torch.bfloat16 else 2.0**-10
    a, b = low.molecule_map.float(), ref.molecule_map
    assert torch.isfinite(a).all() and (a >= 0).all()
    assert ((a - b).abs() <= 8 * eps * b.abs() + 1e-3).float().mean() > 0.999
    # cells integrate from the rounded map values; the damping decisions can then flip in a few
    ca, cb = low.cell_molecules, ref.cell_molecules
    assert torch.isclose(ca, cb, rtol=0.05, atol=0.05).all(dim=1).float().mean() > 0.95


def test_bf16_map_world_round_trips_checkpoint(tmp_path):
    w = ms.World(chemistry=CHEMISTRY, map_size=64, device="cuda", seed=3, map_dtype=torch.bfloat16)
    w.spawn_cells(gen_genomes(100, 400))
    w.enzymatic_activity()
    w.diffuse_molecules()
    w.save_state(tmp_path / "s0")
    mm = w.molecule_map.clone()
    w.diffuse_molecules()
    w.load_state(tmp_path / "s0")
    assert w.molecule_map.dtype == torch.bfloat16 and torch.equal(w.molecule_map, mm)


def test_permeation_matches_host():
    wc = _world("cpu", n=300)
    wg = _copy_world_cpu_to_gpu(wc)
    from magicsoup_amd.ops import world_ops

    world_ops.permeate(wc)
    world_ops.permeate(wg)
    assert torch.allclose(wg.cell_molecules.cpu(), wc.cell_molecules, rtol=1e-6, atol=1e-6)
    assert torch.allclose(wg.molecule_map.cpu(), wc.molecule_map, rtol=1e-6, atol=1e-6)


def _torch_diffuse_permeate(w, mm: torch.Tensor, cm: torch.Tensor, pos: torch.Tensor):
    """The reference's diffuse_molecules (world.py:627-665) in plain fp32 torch on the GPU: one
    circular Conv2d per molecule with the mass correction and clamp, then permeation between each
    cell and its pixel. Independent of the host core."""
    import torch.nn.functional as F

    S = mm.size(1)
    mm = mm.clone()
    for i, (a, b) in enumerate(w._diffusion):
        k = torch.tensor([[a, a, a], [a, b, a], [a, a, a]], dtype=torch.float32, device=mm.device).view(1, 1, 3, 3)
        x = mm[i].view(1, 1, S, S)
        before = x.sum()
        y = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="circular"), k).view(S, S)
        y = y + (before - y.sum()) / (S * S)
        mm[i] = y.clamp(min=0.0)
    m = w.n_molecules
    X = torch.cat([cm, mm[:, pos[:, 0], pos[:, 1]].T], dim=1)
    for i, p in enumerate(w._permeation):
        d_int = X[:, i] * p
        d_ext = X[:, i + m] * p
        X[:, i] += d_ext - d_int
        X[:, i + m] += d_int - d_ext
    mm[:, pos[:, 0], pos[:, 1]] = X[:, m:].T
    return mm, X[:, :m]


@pytest.mark.parametrize("size", [64, 255, 1000])
def test_diffusion_and_permeation_match_torch_conv_oracle(size):
    """World.diffuse_molecules (register-sliding stencil, deferred mass correction, permeation
    kernel) against the reference's torch ops directly on the GPU -- the oracle the host core is
    checked against on the CPU (tests/test_world.py), so the GPU path is pinned independently."""
    w = _world("cuda", map_size=size, n=min(400, size * size // 8))
    w.synchronize()
    pos = w.cell_positions.long()
    mm, cm = _torch_diffuse_permeate(w, w.molecule_map.float(), w.cell_molecules.clone(), pos)
    w.diffuse_molecules()
    got_mm, got_cm = w.molecule_map.float(), w.cell_molecules
    # (summation orders differ: the conv's reduction tree vs the stencil's and the correction's)
    assert torch.allclose(got_mm, mm, rtol=2e-5, atol=2e-5), (got_mm - mm).abs().max()
    assert torch.allclose(got_cm, cm, rtol=2e-5, atol=2e-5), (got_cm - cm).abs().max()
    # and three steps with degradation folded into the stencil (the pending scale)
    for _ in range(3):
        mm = mm * torch.tensor(w._mol_degrads, device="cuda").view(-1, 1, 1)
        cm = cm * torch.tensor(w._mol_degrads, device="cuda").view(1, -1)
        mm, cm = _torch_diffuse_permeate(w, mm, cm, pos)
        w.degrade_molecules()
        w.diffuse_molecules()
    assert torch.allclose(w.molecule_map.float(), mm, rtol=1e-4, atol=1e-4), (w.molecule_map.float() - mm).abs().max()
    assert torch.allclose(w.cell_molecules, cm, rtol=1e-4, atol=1e-4)


def test_neighbors_match_host():
    wc = _world("cpu", map_size=32, n=600)
    wg = _copy_world_cpu_to_gpu(wc)
    idx = list(range(0, wc.n_cells, 2))
    a = set(wc.get_neighbors(idx))
    b = set(wg.get_neighbors(idx))
    assert a == b
    a = set(wc.get_neighbors(idx, nghbr_idxs=list(range(wc.n_cells))))
    b = set(wg.get_neighbors(idx, nghbr_idxs=list(range(wc.n_cells))))
    assert a == b


def _check_invariants(w):
    n = w.n_cells
    assert int(w.cell_map.sum().item()) == n
    pos = w.cell_positions.long()
    keys = pos[:, 0] * w.map_size + pos[:, 1]
    assert keys.unique().numel() == n
    assert bool(w.cell_map[pos[:, 0], pos[:, 1]].all())
    assert len(w.cell_genomes) == n and len(w.cell_labels) == n
    assert w.kinetics.N.size(0) == n


def test_world_lifecycle_on_gpu():
    w = _world("cuda", map_size=64, n=1000)
    _check_invariants(w)
    total0 = w.molecule_map.double().sum(dim=[1, 2]) + w.cell_molecules.double().sum(0)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(5):
        w.enzymatic_activity()
        kill = torch.argwhere(w.cell_molecules[:, atp] < 1.0).flatten()
        w.kill_cells(kill)
        _check_invariants(w)
        repl = torch.argwhere(w.cell_molecules[:, atp] > 5.0).flatten()
        w.cell_molecules[repl, atp] -= 4.0
        w.divide_cells(repl)
        _check_invariants(w)
        w.recombinate_cells(p=1e-4)
        w.mutate_cells(p=1e-4)
        w.degrade_molecules()
        w.diffuse_molecules()
        w.increment_cell_lifetimes()
        w.move_cells()
        _check_invariants(w)
    assert torch.isfinite(w.molecule_map).all() and torch.isfinite(w.cell_molecules).all()
    # re-translating every genome from scratch reproduces the incrementally maintained params
    N = w.kinetics.N.clone()
    w.update_cells([(g, i) for i, g in enumerate(w.cell_genomes)])
    P = min(N.size(1), w.kinetics.N.size(1))
    assert torch.equal(N[:, :P], w.kinetics.N[:, :P])
    del total0


def test_spawn_divide_kill_conserve_mass_on_gpu():
    w = ms.World(chemistry=CHEMISTRY, map_size=128, device="cuda")
    exp = w.molecule_map.double().sum(dim=[1, 2])
    idxs = w.spawn_cells(gen_genomes(1000, 500))
    got = w.molecule_map.double().sum(dim=[1, 2]) + w.cell_molecules.double().sum(0)
    assert torch.all((got - exp).abs() < 1e-1)
    pc = w.divide_cells(idxs)
    got = w.molecule_map.double().sum(dim=[1, 2]) + w.cell_molecules.double().sum(0)
    assert torch.all((got - exp).abs() < 1e-1)
    w.kill_cells(idxs + [c for _, c in pc])
    got = w.molecule_map.double().sum(dim=[1, 2]) + w.cell_molecules.double().sum(0)
    assert torch.all((got - exp).abs() < 1e-1)
    assert w.n_cells == 0


def test_mutations_on_gpu_change_genomes():
    w = _world("cuda", n=500, s=200)
    before = list(w.cell_genomes)
    w.mutate_cells(p=0.01)
    after = list(w.cell_genomes)
    changed = sum(a != b for a, b in zip(before, after))
    assert changed > 300
    w.mutate_cells(p=0.05, p_indel=1.0, p_del=1.0)
    assert all(len(g) <= len(b) for g, b in zip(w.cell_genomes, after))


@pytest.mark.parametrize("mode", [0, 128])
def test_integrator_split_parts_match_fused(mode):
    """The launches a domain-decomposed world uses (flags all-reduced across ranks) reproduce the
    fused single launch exactly: the speculative protocol (one all-reduce of the 12 speculative
    flags + unfit word, then the per-part flags of the exact launches) and, with the speculation
    off (mode bit 7), the plain per-part protocol."""
    from magicsoup_amd.ops import native

    wa = _world("cuda", n=500)
    wa2 = copy.deepcopy(wa)  # (GPU placement is race-resolved: clone rather than rebuild)
    calls = []
    wa2.__dict__["_allreduce_flags"] = lambda flags: calls.append(int(flags.numel()))
    native.hip().set_integrate_mode(mode)
    try:
        wa.enzymatic_activity()
        wa2.enzymatic_activity()
    finally:
        native.hip().set_integrate_mode(0)
    assert calls == ([13, 4, 4, 4] if mode == 0 else [4, 4, 4])
    assert torch.equal(wa.cell_molecules, wa2.cell_molecules)
    assert torch.equal(wa.molecule_map, wa2.molecule_map)


def test_neighbor_slots_match_pair_list():
    w = _world("cuda", map_size=32, n=700)
    from magicsoup_amd.ops import hip_ops

    keys = hip_ops.neighbor_slot_keys(w)
    keys = keys[keys >= 0]
    got = {(int(k) >> 32, int(k) & 0xFFFFFFFF) for k in keys.tolist()}
    assert len(got) == int(keys.numel())  # each pair once
    assert got == set(w.get_neighbors(list(range(w.n_cells))))


def test_param_row_storage_fuzz_matches_dense_model():
    """Random kill / grow / copy / build sequences on GPU row storage (slot map, freed-row reuse,
    packed integrator layout) against a dense cell-ordered model of the same operations."""
    import random as _r

    from magicsoup_amd.ops import kinetics_ops

    rng = _r.Random(5)
    w = _world("cuda", map_size=64, n=120)
    kin = w.kinetics
    names = ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")
    model = {k: getattr(kin, k).clone() for k in names}
    X = torch.rand(kin.N.size(0), kin.N.size(2), device="cuda") * 5
    for step in range(60):
        n = kin.__dict__["_ncells"]
        op = rng.choice(["kill", "grow", "copy", "integrate", "widen", "unset"])
        if op == "kill" and n > 10:
            keep = torch.rand(n, device="cuda") > 0.3
            kin.remove_cell_params(keep)
            for k in names:
                model[k] = model[k][keep]
            X = X[keep]
        elif op == "grow":
            k_new = rng.randint(1, 40)
            kin.increase_max_cells(k_new)
            for k in names:
                z = torch.zeros(k_new, *model[k].shape[1:], dtype=model[k].dtype, device="cuda")
                model[k] = torch.cat([model[k], z])
            X = torch.cat([X, torch.rand(k_new, X.size(1), device="cuda") * 5])
        elif op == "unset" and n > 4:
            # cells sharing a row with others (after "copy") must not clear their sharers
            cells = torch.randperm(n, device="cuda")[: n // 5]
            kin.unset_cell_params(cells)
            for k in names:
                model[k][cells] = 0
        elif op == "widen":
            # protein dimension grows in place of the row storage (slot map kept)
            p_new = kin.N.size(1) + rng.randint(1, 3) if kin.__dict__["_slot"] is None else kin._P() + rng.randint(1, 3)
            kin.increase_max_proteins(p_new)
            for k in names:
                t = model[k]
                if t.dim() >= 2 and t.size(1) < p_new:
                    z = torch.zeros(t.size(0), p_new - t.size(1), *t.shape[2:], dtype=t.dtype, device="cuda")
                    model[k] = torch.cat([t, z], dim=1)
        elif op == "copy" and n > 4:
            src = torch.randperm(n, device="cuda")[: n // 4]
            dst = torch.randperm(n, device="cuda")[: n // 4]
            kin.copy_cell_params(src, dst)
            for k in names:
                model[k][dst] = model[k][src]
        else:
            # integrate through the slot map + packed layout; compare with a dense copy
            dense = Kinetics.__new__(Kinetics)
            dense.__dict__.update(kin.__dict__)
            dense.__dict__.update(_store_d={k: model[k].clone() for k in names}, _slot=None, _hip_scratch=None,
                                  _ncells=model["N"].size(0), _nrows=model["N"].size(0), _packed_stamp=None,
                                  _spare={}, _compact=False)
            dense.__dict__.pop("_hip_scratch")
            Xa, Xb = X.clone(), X.clone()
            kinetics_ops.integrate(kin, Xa, (0.7, 0.2, 0.1), 4)
            kinetics_ops.integrate(dense, Xb, (0.7, 0.2, 0.1), 4)
            assert torch.equal(Xa, Xb), step
    for k in names:
        assert torch.equal(getattr(kin, k), model[k]), k


@pytest.mark.parametrize("n", [1, 63, 4096, 4097, 50_000, 1_000_003])
def test_select_matches_nonzero(n):
    """select.hip compaction (both lists, count and max via pinned memory) against torch.nonzero."""
    from magicsoup_amd.ops import hip_ops

    g = torch.Generator(device="cuda").manual_seed(n)
    mask = torch.rand(n, device="cuda", generator=g) < 0.3
    sel, rest, _ = hip_ops.select(mask, "set", rest=True)
    assert torch.equal(sel, torch.nonzero(mask).flatten())
    assert torch.equal(rest, torch.nonzero(~mask).flatten())
    sel2, _, _ = hip_ops.select(mask, "clear")
    assert torch.equal(sel2, rest)
    v = torch.randint(-5, 6, (n,), dtype=torch.int32, device="cuda", generator=g)
    vals = torch.randint(0, 1000, (n,), dtype=torch.int32, device="cuda", generator=g)
    sel3, _, mx = hip_ops.select(v, "i32pos", vals=vals)
    ref = torch.nonzero(v > 0).flatten()
    assert torch.equal(sel3, ref)
    assert mx == (int(vals[ref].max()) if ref.numel() else 0)
    r = torch.randint(-3, 3, (n,), dtype=torch.int64, device="cuda", generator=g)
    assert torch.equal(hip_ops.select(r, "i64nonneg")[0], torch.nonzero(r >= 0).flatten())


@pytest.mark.parametrize("n", [1, 63, 4097, 50_000, 1_000_003, 4096 * 1024 + 5])
def test_select_async_single_pass_matches_nonzero(n):
    """select_indices_async: the single-pass form (tile counts tagged with a per-call generation,
    select_lb.h; up to 1024 tiles) and the count + write pair (beyond, or switched off) give
    torch.nonzero's lists and count, also for back-to-back calls on the same tile words."""
    from magicsoup_amd.ops import hip_ops, native

    g = torch.Generator(device="cuda").manual_seed(n)
    try:
        for single in (1, 0, 1):
            native.hip().set_select_single_pass(single)
            for p in (0.3, 0.97, 0.0):
                mask = torch.rand(n, device="cuda", generator=g) < p
                sel, rest, dcount, slot = hip_ops.select_async(mask, "set", rest=True)
                cnt = hip_ops.wait_count(slot)
                ref = torch.nonzero(mask).flatten()
                assert cnt == ref.numel() == int(dcount[0])
                assert torch.equal(sel[:cnt], ref)
                assert torch.equal(rest[: n - cnt], torch.nonzero(~mask).flatten())
    finally:
        native.hip().set_select_single_pass(1)


@pytest.mark.parametrize("map_size,n", [(64, 2500), (256, 6_000), (1024, 50_000)])
def test_placement_tail_kernel_matches_all_grid_rounds(map_size, n):
    """The one-barrier placement (round 0 over the grid, later rounds in one workgroup over round 0's
    losers: world.hip place_tail_coop_kernel) places every cell where the all-grid rounds do -- on a
    dense map (long tail) and a sparse one -- for divisions over a mask and for moves."""
    from magicsoup_amd.ops import native

    base = _world("cuda", map_size=map_size, n=n, s=200, seed=5)
    base.synchronize()
    out = []
    try:
        for tail in (1, 0):
            native.hip().set_place_tail(tail)
            w = copy.deepcopy(base)
            ms.set_seed(9)
            w.divide_cells(torch.arange(w.n_cells, device="cuda"))
            w.move_cells(torch.arange(0, w.n_cells, 3, device="cuda"))
            w.synchronize()
            w.check_invariants()
            out.append((w.n_cells, w.cell_positions.clone(), w.cell_map.clone()))
    finally:
        native.hip().set_place_tail(1)
    assert out[0][0] == out[1][0] > n
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][2], out[1][2])


@pytest.mark.parametrize("n", [500, 6_000])
def test_divide_placement_both_paths_keep_occupancy_consistent(n):
    """Single-workgroup placement rounds (k <= 2048) and the multi-launch path (larger k) both
    leave one cell per pixel, children in a parent's Moore neighbourhood and cell_map in sync."""
    w = _world("cuda", map_size=256, n=n, s=200)
    par, chi = w.divide_cells_t(torch.arange(w.n_cells, device="cuda"))
    assert par.numel() > 0.5 * n
    pos = w.cell_positions.long()
    key = pos[:, 0] * 256 + pos[:, 1]
    assert torch.unique(key).numel() == w.n_cells
    assert int(w.cell_map.sum()) == w.n_cells
    d = (pos[par] - pos[chi]).abs()
    d = torch.minimum(d, 256 - d)
    assert bool((d.max(dim=1).values == 1).all())


@pytest.mark.parametrize("n", [500, 6_000, 30_000])
@pytest.mark.parametrize("how", ["list", "mask"])
def test_cooperative_placement_matches_multi_launch_rounds(n, how):
    """The single cooperative launch (grid barriers, early exit) places exactly like the per-round
    launches (same bids, priorities and RNG streams), for index lists and for masks (divide_cells
    with a boolean mask places over the mask without compacting it first)."""
    out = []
    # spawn placement is not deterministic (racing pixel claims): both modes start from one state
    base = _world("cuda", map_size=512 if n > 6000 else 256, n=n, s=100)
    sel = torch.rand(base.n_cells, device="cuda") < 0.7
    for mode in (1, 0):
        w = copy.deepcopy(base)
        arg = sel if how == "mask" else torch.nonzero(sel).flatten()
        native.hip().set_place_mode(mode)
        try:
            ms.set_seed(99)
            par, chi = w.divide_cells_t(arg)
        finally:
            native.hip().set_place_mode(0)
        out.append((par.cpu(), w.cell_positions.cpu().clone(), w.cell_map.cpu().clone()))
        pos = w.cell_positions.long()
        side = w.map_size
        assert torch.unique(pos[:, 0] * side + pos[:, 1]).numel() == w.n_cells
        assert int(w.cell_map.sum()) == w.n_cells
        assert par.numel() > 0.3 * n
    # same items (list positions / cell indices over the mask) -> same RNG streams and priorities:
    # bit-identical placements
    if True:
        assert torch.equal(out[0][0], out[1][0])
        assert torch.equal(out[0][1], out[1][1])
        assert torch.equal(out[0][2], out[1][2])


def test_recombination_commit_on_gpu():
    """Fused recombination commit: disjoint pairs conserve their total length; a cell in several
    pairs keeps one of its results; arena lengths match the materialised strings."""
    from magicsoup_amd.ops import hip_ops

    w = _world("cuda", map_size=64, n=200, s=300)
    before = list(w.cell_genomes)
    pairs = torch.tensor([[2 * i, 2 * i + 1] for i in range(50)], dtype=torch.int32, device="cuda")
    changed = hip_ops.recombinations(w, pairs, 1e-2)
    assert changed.numel() > 0
    after = list(w.cell_genomes)
    for a, b in pairs.tolist():
        assert len(after[a]) + len(after[b]) == len(before[a]) + len(before[b])
    assert sorted(set(changed.tolist())) == sorted(changed.tolist())
    # overlapping pairs (cell 0 in many): committed rows are unique, strings well-formed
    pairs2 = torch.tensor([[0, j] for j in range(1, 40)], dtype=torch.int32, device="cuda")
    ch2 = hip_ops.recombinations(w, pairs2, 1e-2)
    assert torch.unique(ch2).numel() == ch2.numel()
    g = list(w.cell_genomes)
    assert all(set(x) <= set("TCGA") for x in g)
    lens = w._genomes.lens[: w.n_cells].tolist()
    assert lens == [len(x) for x in g]
    w.recombinate_cells(p=1e-3)
    w.mutate_cells(p=1e-3)
    g = list(w.cell_genomes)
    assert w._genomes.lens[: w.n_cells].tolist() == [len(x) for x in g]


def test_deferred_diffusion_correction_matches_materialised():
    """The diffusion correction left pending (read through by the pixel kernels) gives the same
    trajectory as applying it right after every diffusion."""
    import copy as _copy

    a = _world("cuda", map_size=96, n=400, s=400)
    a.molecule_map = a.molecule_map * 0.01  # near-zero pixels so that the clamp also matters
    b = _copy.deepcopy(a)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for step in range(6):
        for w, eager in ((a, False), (b, True)):
            ms.set_seed(100 + step)
            w.enzymatic_activity()
            w.kill_cells(w.cell_molecules[:, atp] < 0.5)
            w.spawn_cells([ms.random_genome(300) for _ in range(5)])
            w.degrade_molecules()
            w.diffuse_molecules()
            if eager:
                _ = w.molecule_map  # materialise now
        assert a.__dict__["_pending_corr"] is not None
    assert a.n_cells == b.n_cells
    assert torch.allclose(a.molecule_map, b.molecule_map, rtol=1e-5, atol=1e-6)
    assert torch.allclose(a.cell_molecules, b.cell_molecules, rtol=1e-5, atol=1e-6)
    assert float(a.molecule_map.min()) >= 0.0


def _genetics_run(monkeypatch, base, sync: bool, d_cap=None, steps=5, mut_kw=None, rec_p=1e-4, prep=None):
    import copy as _copy

    from magicsoup_amd.ops import genome_pipeline

    if sync:
        monkeypatch.setenv("MS_SYNC_GENETICS", "1")
    else:
        monkeypatch.delenv("MS_SYNC_GENETICS", raising=False)
    if d_cap is not None:
        monkeypatch.setattr(genome_pipeline, "D_CAP", d_cap)
    w = _copy.deepcopy(base)  # identical start (GPU spawn placement is claim-order dependent)
    if prep is not None:
        prep(w)
    ms.set_seed(11)
    torch.manual_seed(11)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for _ in range(steps):
        w.enzymatic_activity()
        w.kill_cells(w.cell_molecules[:, atp] < 0.3)
        w.divide_cells_t(w.cell_molecules[:, atp] > 3.0)
        w.recombinate_cells(p=rec_p)
        w.mutate_cells(**(mut_kw or {"p": 1e-3}))
        w.diffuse_molecules()
    w.enzymatic_activity()
    names = ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")
    params = {k: getattr(w.kinetics, k).clone() for k in names}
    from magicsoup_amd.ops import world_ops

    params["_nprot"] = world_ops.translate(w, torch.arange(w.n_cells, device=w.device))[1]
    return list(w.cell_genomes), params, w.cell_molecules.clone()


def _real(p: dict) -> dict:
    return {k: v for k, v in p.items() if not k.startswith("_")}


def _assert_params_equal(p0: dict, p1: dict, nprot: torch.Tensor) -> None:
    """Parameters of two runs agree on every real protein (p < the cell's protein count); padding
    slots are inert in both (no stoichiometry, no Vmax). Padding Km / Ke values depend on history,
    as in the reference: a widened layout is zero-filled, a build writes the values of an empty
    protein (kinetics.py:577-625 over the batch's protein dimension)."""
    for k in p0:
        a, b = p0[k], p1[k]
        P = min(a.size(1), b.size(1))
        real = torch.arange(P, device=a.device)[None, :] < nprot.to(a.device)[:, None]
        m = real if a.dim() == 2 else real[:, :, None].expand(-1, -1, a.size(2))
        assert torch.equal(a[:, :P][m], b[:, :P][m]), k
        if k in ("N", "Nf", "Nb", "A", "Vmax"):
            for t in (a, b):
                assert not t[:, :P][~m].any() and not t[:, P:].any(), k


def test_device_genome_pipeline_arena_overflow_replay(monkeypatch):
    """Genomes exactly as wide as the arena rows, insertion-only mutations and frequent
    recombination: results that do not fit the arena are committed at reconcile (width flag) and
    the calls queued behind them are replayed (skipped flag) -- same genomes, parameters and
    trajectory as the synchronous path."""
    from magicsoup_amd.ops import genome_pipeline

    seen = []
    orig = genome_pipeline.reconcile

    def spy(world):
        st = world.__dict__.get("_gp_state")
        if st and st["pending"]:
            st["pending"][-1].event.synchronize()
            for pd in st["pending"]:
                seen.append(int(pd.host[1]))
                if pd.kind == "evo":  # (a merged recombinate + mutate call: the halves' flags)
                    seen.extend(int(pd.replay[h].host[1]) for h in ("rec", "mut"))
        orig(world)


    def tighten(w):
        # the genome pool's length bound exactly at the longest genome: longer results are committed
        # at reconcile (width flag) and the calls queued behind them replayed (skipped flag)
        w._genomes.width = 512
        assert int(w._genomes.lens[: w._genomes.n].max()) <= 512

    base = _world("cuda", map_size=64, n=0, seed=5)
    base.spawn_cells([ms.random_genome(512) for _ in range(600)])
    assert int(base._genomes.lens[: base.n_cells].max()) == 512
    kw = dict(steps=3, mut_kw={"p": 1.5e-3, "p_indel": 1.0, "p_del": 0.0}, rec_p=2e-4, prep=tighten)
    g0, p0, x0 = _genetics_run(monkeypatch, base, sync=True, **kw)
    monkeypatch.setattr(genome_pipeline, "reconcile", spy)
    g1, p1, x1 = _genetics_run(monkeypatch, base, sync=False, **kw)
    assert any(f & genome_pipeline._F_WIDTH for f in seen), seen
    assert any(f & genome_pipeline._F_SKIPPED for f in seen), seen
    assert g0 == g1
    _assert_params_equal(_real(p0), _real(p1), p0["_nprot"])
    assert torch.equal(x0, x1)


def test_device_genome_pipeline_capacity_skip_replays(monkeypatch):
    """Capacities far below the selected counts: every call turns into a no-op that reconcile
    replays on the synchronous path -- same result as that path."""
    from magicsoup_amd.ops import genome_pipeline

    base = _world("cuda", map_size=64, n=800, s=400, seed=7)
    g0, p0, x0 = _genetics_run(monkeypatch, base, sync=True, steps=3)
    monkeypatch.setattr(genome_pipeline, "_cap", lambda expected, limit: 2)
    g1, p1, x1 = _genetics_run(monkeypatch, base, sync=False, steps=3)
    assert g0 == g1
    _assert_params_equal(_real(p0), _real(p1), p0["_nprot"])
    assert torch.equal(x0, x1)


@pytest.mark.parametrize("d_cap", [None, 1, 4, "p6", "blob"])
def test_device_genome_pipeline_matches_sync_path(monkeypatch, d_cap):
    """Sync-free mutate / recombinate (device counts, speculative token layout, fresh rows) give
    the same genomes, parameters and trajectory as the synchronous path; with one domain slot
    or four per protein the cells past the layout are listed and rebuilt alone at reconcile (gp.hip
    overflow list; every changed cell once the list overflows) -- same result."""
    from magicsoup_amd.ops import genome_pipeline

    base = _world("cuda", map_size=64, n=800, s=400, seed=7)
    kw = {}
    if d_cap == "p6":  # (six protein slots per cell in the chain's layout: larger proteomes listed)
        monkeypatch.setattr(genome_pipeline, "P_CAP", 6)
        d_cap = 12
    blob = d_cap == "blob"
    if blob:  # (no call fits the scratch bound: every one declines to the synchronous path)
        monkeypatch.setattr(genome_pipeline, "_BLOB_MAX", 1)
        d_cap = None
    if d_cap == 4:  # (genomes past the LDS slots: the chain's global-slot pass, a workgroup each;
        # the rate keeps rate * length bound within genome_pipeline.LAM_MAX)
        ms.set_seed(4)
        base.spawn_cells([ms.random_genome(n) for n in (2100, 2500, 3000, 3500, 4000)])
        kw = dict(mut_kw={"p": 2e-4})
    g0, p0, x0 = _genetics_run(monkeypatch, base, sync=True, **kw)
    seen = []
    orig = genome_pipeline._rebuild_set

    def spy(pd):
        seen.append(int(pd.host[1]))
        return orig(pd)

    monkeypatch.setattr(genome_pipeline, "_rebuild_set", spy)
    g1, p1, x1 = _genetics_run(monkeypatch, base, sync=False, d_cap=d_cap, **kw)
    if blob:
        assert not seen, seen
    if d_cap is not None:  # (listed cells, or every changed cell once the list overflowed)
        assert any(f & (genome_pipeline._F_PARTIAL | genome_pipeline._F_TRANSLATE) for f in seen), seen
    assert g0 == g1
    _assert_params_equal(_real(p0), _real(p1), p0["_nprot"])
    assert torch.equal(x0, x1)


@pytest.mark.parametrize("mode", ["plain", "overflow", "capacity", "dcap"])
def test_merged_recombinate_mutate_chain_matches_separate_calls(monkeypatch, mode):
    """recombinate_cells() + mutate_cells() queued back to back run as one device chain with one
    rebuild of the union of changed cells (genome_pipeline.evolve, gp.hip gp_evolve): same genomes,
    parameters and trajectory as two separate pipeline calls -- also when results outgrow the arena
    (re-commit + replay), when the selections exceed the call capacities (replay of both halves), and
    when proteomes exceed the token slots (union rebuilt on the host)."""
    import magicsoup_amd.models.world as world_mod
    from magicsoup_amd.ops import genome_pipeline

    calls = []
    orig = genome_pipeline.evolve

    def spy(world, *a, **kw):
        ok = orig(world, *a, **kw)
        calls.append(ok)
        return ok

    def tighten(w):
        w._genomes.width = 512

    # (mutation rate * genome length bound <= genome_pipeline.LAM_MAX keeps the mutations on the pipeline;
    # recombination at 5e-5 keeps the pair capacity's gate -- 8 n p L <= N_CAP, with lengths doubling
    # where pairs recombine -- out of reach within the 4 steps whatever the start; the world is
    # seeded, so the start does not depend on the tests that ran before)
    import random

    random.seed(17)
    ms.set_seed(17)
    torch.manual_seed(17)
    kw = dict(steps=4, mut_kw={"p": 2e-4}, rec_p=5e-5)
    if mode == "overflow":
        base = _world("cuda", map_size=64, n=0, seed=5)
        base.spawn_cells([ms.random_genome(512) for _ in range(600)])
        kw.update(mut_kw={"p": 1.5e-3, "p_indel": 1.0, "p_del": 0.0}, rec_p=2e-4, prep=tighten)
    else:
        base = _world("cuda", map_size=64, n=800, s=400, seed=7)
    if mode == "capacity":
        monkeypatch.setattr(genome_pipeline, "_cap", lambda expected, limit: 2)
    d_cap = 1 if mode == "dcap" else None
    monkeypatch.setattr(world_mod.World, "_evolve", lambda self, *a: 0)
    g0, p0, x0 = _genetics_run(monkeypatch, base, sync=False, d_cap=d_cap, **kw)
    monkeypatch.undo()
    if mode == "capacity":
        monkeypatch.setattr(genome_pipeline, "_cap", lambda expected, limit: 2)
    monkeypatch.setattr(genome_pipeline, "evolve", spy)
    g1, p1, x1 = _genetics_run(monkeypatch, base, sync=False, d_cap=d_cap, **kw)
    # the merged chain ran (every step; with results outgrowing the bound, until the bound grew
    # past what the mutation rate allows on the device pipeline)
    assert any(calls) and (all(calls) or mode == "overflow"), calls
    assert g0 == g1
    _assert_params_equal(_real(p0), _real(p1), p0["_nprot"])
    assert torch.equal(x0, x1)


def test_assignment_after_speculative_activity_survives_rollback(monkeypatch):
    """A speculative enzymatic_activity (issued on top of unconfirmed genome-pipeline rebuilds)
    whose rebuilds must be redone on the host is rolled back and re-run at the next confirmation.
    Assigning ``cell_molecules`` / ``molecule_map`` confirms it first, so the user's values are what
    the world holds afterwards (one domain slot per protein forces the host rebuild)."""
    from magicsoup_amd.ops import genome_pipeline

    monkeypatch.delenv("MS_SYNC_GENETICS", raising=False)
    monkeypatch.setattr(genome_pipeline, "D_CAP", 1)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for target in ("cell_molecules", "molecule_map"):
        w = _world("cuda", map_size=64, n=600, s=500, seed=5)
        for _ in range(2):  # parameter storage and the pipeline are set up
            w.enzymatic_activity()
            w.kill_cells(w.cell_molecules[:, atp] < 0.3)
            w.divide_cells_t(w.cell_molecules[:, atp] > 3.0)
            w.diffuse_molecules()
        w.recombinate_cells(p=1e-4)
        w.mutate_cells(p=2e-4)  # queued / pending device-pipeline rebuilds (p * row width <= 1)
        w.enzymatic_activity()
        st = w.__dict__.get("_gp_state")
        assert w.__dict__.get("_spec") is not None, (st, w.__dict__.get("_deferred"))
        x = torch.full_like(w.__dict__["_molmap"] if target == "molecule_map" else w._cols[target].view(w.n_cells), 3.0)
        setattr(w, target, x.clone())
        assert w.__dict__.get("_spec") is None
        assert torch.equal(getattr(w, target), x), target


def test_deferred_genome_ops_match_immediate_issue(monkeypatch):
    """All-cells mutate / recombinate go to a side stream (issued at once and joined at the next op
    that needs them, or queued until the diffusion stencil is launched): same genomes, parameters and
    trajectory as issuing them on the compute stream; reading ``cell_genomes`` confirms them."""
    import magicsoup_amd.models.world as world_mod

    base = _world("cuda", map_size=64, n=800, s=400, seed=7)
    monkeypatch.setattr(world_mod, "_DEFER_ENV", "0")
    g0, p0, x0 = _genetics_run(monkeypatch, base, sync=False)
    monkeypatch.setattr(world_mod, "_DEFER_ENV", "1")
    g1, p1, x1 = _genetics_run(monkeypatch, base, sync=False)
    assert g0 == g1
    _assert_params_equal(_real(p0), _real(p1), p0["_nprot"])
    assert torch.equal(x0, x1)
    # default: queued until the diffusion
    w = copy.deepcopy(base)
    w.recombinate_cells(p=1e-4)
    w.mutate_cells(p=1e-3)
    w.degrade_molecules()
    assert len(w.__dict__.get("_deferred", [])) == 2
    w.diffuse_molecules()
    assert not w.__dict__["_deferred"]
    genomes = list(w.cell_genomes)
    assert not w.__dict__.get("_gp_state", {}).get("pending") and len(genomes) == w.n_cells


def test_widening_proteins_keeps_parameters_in_slot_mode():
    """Growing the protein dimension while cells map to scattered (collected, shared) ragged records
    moves nothing: every cell keeps its parameters, the new protein slots read as zeros."""
    import bench

    atp = CHEMISTRY.molname_2_idx["ATP"]
    w = _world("cuda", map_size=96, n=1500, s=500)
    for _ in range(4):
        bench.step(w, 1500, 500, atp)
        w.mutate_cells(p=1e-4)
    w._reconcile()
    kin = w.kinetics
    kin._collect_records(0)  # (records compacted; later builds take fresh ones past them)
    bench.step(w, 1500, 500, atp)
    w.mutate_cells(p=1e-4)
    w._reconcile()
    assert kin.__dict__["_slot"] is not None
    names = ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")
    # dense copies through the public tensors (a clone of the world keeps the original's layout)
    ref = copy.deepcopy(w)
    before = {k: getattr(ref.kinetics, k).clone() for k in names}
    P = kin._P()
    kin.increase_max_proteins(P + 7)
    assert kin._P() == P + 7
    for k in names:
        t = getattr(kin, k)
        assert torch.equal(t[:, :P], before[k]), k
        assert not t[:, P:].any(), k
    w.enzymatic_activity()
    ref.enzymatic_activity()
    assert torch.equal(w.cell_molecules, ref.cell_molecules)


def _integrate_modes(kin, X, modes=(0, 8)):
    from magicsoup_amd.ops import kinetics_ops

    out = {}
    try:
        for mode in modes:
            native.hip().set_integrate_mode(mode)
            Xk = X.clone()
            kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), 4)
            out[mode] = Xk
    finally:
        native.hip().set_integrate_mode(0)
    return out


@pytest.mark.parametrize("case", ["wl500", "wl3000", "wl8000", "syn20", "syn40", "syn64", "big_exponents",
                                  "syn64_big_exponents"])
def test_register_integrator_matches_lds_integrator_bit_for_bit(case):
    """The register-resident launches (mode 0: cells with <= 32 / 64 active proteins and <= 16
    non-zero signals per protein; the rest through a 64-lane launch with 32 non-zeros per protein,
    and what does not fit there through the wide LDS launch; mode 32 skips the 64-lane level)
    against the legacy LDS-staged launches (mode 8) on the same state: identical results, bit for
    bit."""
    if case.startswith("syn"):
        from magicsoup_amd.examples.synthetic import make_chemistry

        m = int(case[3:].split("_")[0])
        chem = make_chemistry(m, 2 * m, seed=3)
    else:
        chem = CHEMISTRY
    ms.set_seed(2)
    torch.manual_seed(2)
    w = ms.World(chemistry=chem, map_size=64, device="cuda", seed=2)
    size = {"wl3000": 3000, "wl8000": 8000}.get(case, 500)
    w.spawn_cells(gen_genomes(300, size))
    kin = w.kinetics
    if case.endswith("big_exponents"):
        # stoichiometries / Hill numbers beyond the branch-free power range (>= 8) in some proteins,
        # and (two signals per lane) beyond its 16-bit entries' exponent range (>= 16)
        Nf, A = kin.Nf.clone(), kin.A.clone()
        Nf[::7, :, 1] = torch.where(Nf[::7, :, 1] > 0, 9, Nf[::7, :, 1])
        Nf[::11, :, 0] = torch.where(Nf[::11, :, 0] > 0, 17, Nf[::11, :, 0])
        A[::5, :, 2] = torch.where(A[::5, :, 2] != 0, -9, A[::5, :, 2])
        kin.Nf, kin.A = Nf, A
    na = (kin.Vmax > 0).sum(1)
    if case == "wl3000":
        assert int(na.max()) > 32  # exercises the wide launch
    if case == "wl8000":
        # multi-group cells beyond two chunks (the speculative launch's wide role: 8 groups of 32)
        assert int(na.max()) > 64 and int(((na > 64) & (na <= 256)).sum()) >= 10
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    out = _integrate_modes(kin, X, modes=(0, 8, 32, 64, 128, 256))
    assert torch.equal(out[256], out[8])
    assert torch.equal(out[0], out[8])
    assert torch.equal(out[32], out[8])
    assert torch.equal(out[64], out[8])
    assert torch.equal(out[128], out[8])
    assert not torch.equal(out[0], X)


def _spec_held(kin, nparts=3, n_iters=4):
    from magicsoup_amd.ops import hip_ops

    w = hip_ops._scratch(kin).bufs["spec"].cpu().tolist()[4:]
    return not w[4 * nparts] and all(w[4 * p + it] for p in range(nparts) for it in range(n_iters))


@pytest.mark.parametrize("case", ["wl3000", "wl20", "syn16", "syn16_few", "wl9000bp", "exp40"])
def test_speculative_integrator_matches_per_part_launches(case):
    """Mode 0 runs all parts in one speculative launch (each part starting from the previous part's
    last candidate) with the exact per-part LDS launches behind it as the fallback; mode 128 runs
    the per-part launches. Same state, same results bit for bit and the same iteration flags, both
    when the speculation holds (thousands of cells) and when it does not (a few cells: some part's
    global loop ends early)."""
    from magicsoup_amd.ops import kinetics_ops

    chem = CHEMISTRY
    if case.startswith("syn"):
        from magicsoup_amd.examples.synthetic import make_chemistry

        chem = make_chemistry(16, 32, seed=3)
    n = {"wl3000": 3000, "syn16": 3000, "wl9000bp": 400, "exp40": 3000}.get(case, 20)
    ms.set_seed(4)
    torch.manual_seed(4)
    w = ms.World(chemistry=chem, map_size=128, device="cuda", seed=4)
    w.spawn_cells(gen_genomes(n, 9000 if case == "wl9000bp" else 500))
    kin = w.kinetics
    if case == "wl9000bp":
        # proteomes beyond the 64-lane slots: the speculative LDS launch takes those cells
        assert int((kin.Vmax > 0).sum(1).max()) > 64
    if case == "exp40":
        # exponents beyond the register paths' 5-bit fields (same route)
        Nf = kin.Nf.clone()
        Nf[::9, :, 2] = torch.where(Nf[::9, :, 2] > 0, 40, Nf[::9, :, 2])
        kin.Nf = Nf
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    res, masks, held = {}, {}, None
    try:
        for mode in (0, 128):
            native.hip().set_integrate_mode(mode)
            Xk = X.clone()
            masks[mode] = kinetics_ops.integrate(kin, Xk, (0.7, 0.2, 0.1), 4)
            res[mode] = Xk
            if mode == 0:
                held = _spec_held(kin)
    finally:
        native.hip().set_integrate_mode(0)
    assert torch.equal(res[0], res[128])
    assert masks[0] == masks[128]
    assert held == (masks[128] == [15, 15, 15])
    if n >= 3000:
        assert held  # the flagship regime: the speculation holds

    # the world path (gather from / scatter to cell molecules and pixels); mode 256: the speculative
    # launches store their states for the write-back kernel instead of writing the world directly
    w2, w3 = copy.deepcopy(w), copy.deepcopy(w)
    try:
        native.hip().set_integrate_mode(128)
        w2.enzymatic_activity()
        native.hip().set_integrate_mode(256)
        w3.enzymatic_activity()
    finally:
        native.hip().set_integrate_mode(0)
    w.enzymatic_activity()
    for x in (w2, w3):
        assert torch.equal(w.cell_molecules, x.cell_molecules)
        assert torch.equal(w.molecule_map, x.molecule_map)


def test_integrator_flags_match_host_core_on_small_populations():
    """The reference's global exit depends on every cell's flags. A cell whose damping factors stop
    changing (its remaining iterations are copies) still repeats an impactful correction that
    changed nothing (a backward reaction with its factor capped at 1), so its flag must stay raised
    in the remaining iterations. Small populations make single cells decide the exit: the device
    integrator (speculative launch, fallback, fixed-point exits) must report the host core's flags
    (which iterates without shortcuts) and its results."""
    base = _world("cpu", n=200, seed=5)
    gen = torch.Generator().manual_seed(5)
    early = close = cells = 0
    for trial in range(24):
        keep = torch.randperm(base.n_cells, generator=gen)[: 1 + trial % 4]
        wc = copy.deepcopy(base)
        drop = torch.ones(wc.n_cells, dtype=torch.bool)
        drop[keep] = False
        wc.kill_cells(torch.nonzero(drop).flatten())
        wg = _copy_world_cpu_to_gpu(wc)
        pos = wc.cell_positions.long()
        X = torch.cat([wc.cell_molecules, wc.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
        Xc = wc.kinetics.integrate_signals(X)
        Xg = wg.kinetics.integrate_signals(X.cuda()).cpu()
        assert wg.kinetics.last_masks == wc.kinetics.last_masks, trial
        close += int(torch.isclose(Xg, Xc, rtol=1e-5, atol=1e-6).all(dim=1).sum())
        cells += wc.n_cells
        early += wc.kinetics.last_masks != [15, 15, 15]
    assert early > 0  # some populations end a part early
    assert close >= 0.95 * cells, (close, cells)  # (rare last-ulp differences, as in the tests above)


@pytest.mark.parametrize("recycle", [False, True])
def test_parameter_rows_follow_genomes_through_bench_steps(monkeypatch, recycle):
    """After kills (the cell -> records map gathered with the columns), divisions (cloned in the same
    gather), mutations / recombinations (device pipeline) and spawns, every cell's parameters equal
    a fresh translation + build of its current genome. ``recycle``: the record pool is declared
    used up midway (device counter at the capacity), so the device chains run out of records (their
    cells are rebuilt on the host) and the next reservation collects the live records."""
    import bench

    recycled = []
    orig = Kinetics._collect_records

    def spy(self, need):
        orig(self, need)
        recycled.append(True)

    monkeypatch.setattr(Kinetics, "_collect_records", spy)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    w = _world("cuda", map_size=128, n=3000, s=500)
    for i in range(8):
        if recycle and i >= 4:
            # every fresh row taken (again each step: a widening of the protein dimension in
            # between re-packs the storage densely with fresh spare rows)
            w._reconcile()
            kin = w.kinetics
            kin.__dict__["_rtop"].fill_(kin._rec_cap() - 8)
            kin.__dict__["_rtop_ub"] = kin._rec_cap() - 8
        bench.step(w, 3000, 500, atp)
        # the step's genome chains were flushed onto the side stream and are joined lazily (at the
        # next activity): compute-stream allocations of storage-sized blocks now must not receive
        # storage the chains' issue replaced (a recycle / growth inside the flush) while they still
        # read it (World._storage_refs keeps it referenced until the join)
        junk = [torch.full_like(t, 3) for t in w.kinetics.__dict__["_store_d"].values()]
        del junk
        w.mutate_cells(p=1e-4)
        w.recombinate_cells(p=1e-5)
    w._reconcile()
    if recycle:
        assert any(recycled), recycled  # (without forcing, recycling may or may not happen in 8 steps)
    ref = copy.deepcopy(w)
    ref._update_params_rows(torch.arange(ref.n_cells, device="cuda"))
    ka, kb = w.kinetics, ref.kinetics
    P = min(ka.N.size(1), kb.N.size(1))
    real = kb.Vmax[:, :P] != 0  # proteins of the current proteomes (padding has Vmax 0)
    assert torch.equal(ka.Vmax[:, :P], kb.Vmax[:, :P])
    assert int(real.sum()) > w.n_cells  # the population does have proteomes
    for name in ("N", "Nf", "Nb", "A", "Kmf", "Kmb", "Ke", "Kmr"):
        ta, tb = getattr(ka, name)[:, :P], getattr(kb, name)[:, :P]
        assert ta.size(0) == tb.size(0) == w.n_cells
        # padding values depend on history (a widened layout is zero-filled, a build writes the
        # reference's padding values, as in the reference): compare the real proteins
        assert torch.equal(ta[real], tb[real]), name


@pytest.mark.parametrize("probe", [None, "n_cells", "cell_positions", "cell_genomes", "kinetics"])
def test_lazy_division_matches_synchronous_division(probe):
    """divide_cells_t(mask, lazy=True) (the bench loop: the reference discards the pairs) leaves the
    winner count pending; the genome ops and degradation are issued against the device state, the
    diffusion adopts the count after its stencil launch, and any earlier read (``probe``) adopts it
    at once. The world evolves bit for bit as with the synchronous division."""
    base = _world("cuda", map_size=64, n=900, s=400, seed=7)
    atp = CHEMISTRY.molname_2_idx["ATP"]

    def run(lazy: bool):
        w = copy.deepcopy(base)
        ms.set_seed(3)
        torch.manual_seed(3)
        sizes = []
        for _ in range(6):
            w.enzymatic_activity()
            w.kill_cells(w.cell_molecules[:, atp] < 1.0)
            repl = w.cell_molecules[:, atp] > 5.0
            w.cell_molecules[:, atp] -= 4.0 * repl
            n_before = w.n_cells
            out = w.divide_cells_t(repl, lazy=lazy)
            if lazy:
                assert out is None and w.__dict__.get("_count_pending") is not None
                if probe == "n_cells":
                    assert w.n_cells >= n_before
                elif probe == "cell_positions":
                    assert w.cell_positions.size(0) == w.n_cells
                elif probe == "cell_genomes":
                    assert len(w.cell_genomes) == w.n_cells
                elif probe == "kinetics":
                    assert w.kinetics.Vmax.size(0) == w.n_cells
                if probe is not None:
                    assert w.__dict__.get("_count_pending") is None
            w.recombinate_cells(p=1e-4)
            w.mutate_cells(p=1e-3)
            w.degrade_molecules()
            if lazy and probe is None:
                assert w.__dict__.get("_count_pending") is not None  # nothing so far needed the count
            w.diffuse_molecules()
            assert w.__dict__.get("_count_pending") is None
            w.increment_cell_lifetimes()
            sizes.append(w.n_cells)
        torch.cuda.synchronize()
        state = {k: getattr(w, k).clone() for k in ("cell_molecules", "cell_positions", "cell_lifetimes",
                                                     "cell_divisions", "molecule_map", "cell_map")}
        state["Vmax"] = w.kinetics.Vmax.clone()
        return sizes, list(w.cell_genomes), state

    s0, g0, st0 = run(False)
    s1, g1, st1 = run(True)
    assert s0 == s1 and g0 == g1
    for k in st0:
        assert torch.equal(st0[k], st1[k]), k


def test_int8_overflow_of_packed_parameters_raises():
    """A stoichiometry outside the integrator's packed int8 layout is reported through the mapped
    host flag (no copy launch): the next integration raises instead of computing with a wrapped
    coefficient."""
    w = _world("cuda", map_size=32, n=60, s=500, seed=4)
    w.enzymatic_activity()
    kin = w.kinetics
    N = kin.N.clone()
    N[0, 0, 0] = 300
    kin.N = N
    with pytest.raises(OverflowError):
        w.enzymatic_activity()
        torch.cuda.synchronize()
        w.enzymatic_activity()


def test_synchronize_settles_pending_work():
    """World.synchronize() (what bench.py stops its clock after): a lazy division's count adopted,
    queued genome ops issued and confirmed, a speculative activity confirmed, the device idle."""
    w = _world("cuda", map_size=64, n=600, s=400, seed=3)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    w.enzymatic_activity()
    w.divide_cells_t(w.cell_molecules[:, atp] > 2.0, lazy=True)
    w.recombinate_cells(p=1e-4)
    w.mutate_cells(p=1e-3)
    w.degrade_molecules()
    w.enzymatic_activity()  # speculative on top of the queued chains
    w.synchronize()
    d = w.__dict__
    assert d.get("_count_pending") is None and not d.get("_deferred") and d.get("_spec") is None
    assert not (d.get("_gp_state") or {}).get("pending")
    assert len(w.cell_genomes) == w.n_cells == w.kinetics.Vmax.size(0)


# ---------------------------------------------------------------------------- genome pool
def test_genome_pool_is_ragged_and_shared():
    """GPU genomes live in one ragged pool (models/strings.py PoolArena): a 20 kbp genome costs
    ~20 kB of pool (no population-wide widening), children share their parent's bytes, kills and
    divisions move offsets only, and a collection keeps every genome (and the sharing) intact."""
    w = _world("cuda", map_size=96, n=2000, s=500)
    g = w._genomes
    assert type(g).__name__ == "PoolArena"
    w._reconcile()
    top0 = g.top_ub = int(g.top.item())
    w.update_cells([(ms.random_genome(20_000), 3)])
    w._reconcile()
    grew = int(g.top.item()) - top0
    assert 20_000 <= grew < 10 << 20, grew
    assert len(w.cell_genomes[3]) == 20_000 and g.width >= 20_000
    # a division: children share their parent's genome storage
    n0 = w.n_cells
    parents, children = w.divide_cells_t(torch.arange(0, 40, device="cuda"))
    assert children.numel() > 0
    assert torch.equal(g.off[children], g.off[parents]) and torch.equal(g.lens[children], g.lens[parents])
    assert w.n_cells == n0 + children.numel()
    # evolve a little, then collect: same genomes, shared genomes still shared, less pool in use
    for _ in range(3):
        w.mutate_cells(p=1e-4)
        w.recombinate_cells(p=1e-5)
        w.kill_cells(torch.arange(0, w.n_cells, 7, device="cuda"))
    before = list(w.cell_genomes)
    w._reconcile()
    used = int(g.top.item())
    off = g.off[: g.n].clone()
    g.collect()
    assert int(g.top.item()) <= used
    assert list(w.cell_genomes) == before
    # cells that shared storage before still do (and only those)
    same_before = off.unsqueeze(0) == off.unsqueeze(1)
    new = g.off[: g.n]
    assert torch.equal(same_before, new.unsqueeze(0) == new.unsqueeze(1))
    g.check()
    w.enzymatic_activity()
    w.check_invariants()


def test_genome_pool_collect_keeps_genomes_next_to_empty_ones():
    """An empty genome still takes a 16-byte allocation (hip_common.h pool_alloc): every allocation
    has an offset of its own, before and after a collection, and the genome allocated right after
    an empty one survives the collection intact."""
    w = _world("cuda", map_size=64, n=200, s=300)
    g = w._genomes
    w._reconcile()
    w.update_cells([("", 5)])
    w.update_cells([(ms.random_genome(700), 6)])
    w._reconcile()
    assert int(g.off[6]) == int(g.off[5]) + 16 and int(g.lens[5]) == 0 and int(g.lens[6]) == 700
    before = list(w.cell_genomes)
    g.collect()
    assert list(w.cell_genomes) == before
    assert int(g.off[5]) != int(g.off[6])


def test_genome_pool_grows_and_collects_under_pressure():
    """A pool too small for what the steps allocate collects / grows on demand (host writes and the
    device pipeline's worst cases are accounted for before any allocation); genomes stay exact."""
    from magicsoup_amd.models import strings

    import bench

    atp = CHEMISTRY.molname_2_idx["ATP"]
    w = _world("cuda", map_size=96, n=1500, s=500)
    g = w._genomes
    w._reconcile()
    g.collect()  # pool exactly as large as the live genomes (plus the minimum)
    cap0 = g.pool_cap
    for _ in range(6):
        bench.step(w, 1500, 500, atp)
        w.mutate_cells(p=2e-4)
        w.update_cells([(ms.random_genome(3000), i) for i in range(0, 60, 3)])
    w._reconcile()
    g.check()
    assert int(g.top.item()) <= g.pool_cap
    assert all(len(x) == int(n) for x, n in zip(w.cell_genomes, g.lens[: g.n].tolist()))
    assert g.pool_cap >= cap0 or strings._POOL_MIN == cap0


@pytest.mark.parametrize("size,cells,dtype", [(2048, 20_000, torch.float32), (12800, 60_000, torch.float16)])
def test_memory_model_matches_a_live_world(size, cells, dtype):
    """utils/memory.py models what a GPU world holds: the modelled footprint of a world after some
    steps is within 25 % of the bytes its tensors hold (utils.memory.measured) and of what the
    caching allocator has handed out. The fp16 case holds a 4.6 GB map (2.3G values: offsets past
    2^31 in every map kernel)."""
    import bench
    from magicsoup_amd.utils import memory

    atp = CHEMISTRY.molname_2_idx["ATP"]
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    w = ms.World(chemistry=CHEMISTRY, map_size=size, device="cuda", seed=3, map_dtype=dtype)
    w.spawn_cells(bench.random_genomes(cells, 500, "cuda"))
    for _ in range(5):
        bench.step(w, cells, 500, atp)
    w.synchronize()
    if size > 8192:
        assert w.molecule_map.numel() > 2**31
        w.check_invariants()
        assert torch.isfinite(w.molecule_map[-1, -64:, -64:].float()).all()
    # (the storage's actual protein dimension: the model's default budgets for recombinants)
    model = memory.footprint(size, len(CHEMISTRY.molecules), w.n_cells, dtype, 500, p_max=w.kinetics._P())["total"]
    held = memory.measured(w)["bytes"]
    alloc = torch.cuda.memory_allocated() - base
    assert 0.75 * held <= model <= 1.25 * held, (model, held)
    assert held <= alloc * 1.05, (held, alloc)


def test_diffusion_past_2_31_map_values():
    """A map of more than 2^31 values (fp16, 14 x 13056^2): the last plane, which starts past 2^31,
    diffuses exactly as a circular 3x3 convolution of its own values (plus the mass correction)."""
    import torch.nn.functional as F

    w = ms.World(chemistry=CHEMISTRY, map_size=13056, device="cuda", seed=4, map_dtype=torch.float16)
    mm = w.molecule_map
    assert mm.numel() > 2**31 and (mm.size(0) - 1) * mm[0].numel() > 2**31
    j = mm.size(0) - 1
    x = mm[j].float().clone()
    a, b = w._diffusion[j]
    w.diffuse_molecules()
    k = torch.full((3, 3), a, device="cuda")
    k[1, 1] = b
    ref = F.conv2d(F.pad(x[None, None], (1, 1, 1, 1), mode="circular"), k[None, None])[0, 0]
    ref = (ref + (x.double().sum() - ref.double().sum()) / x.numel()).clamp(min=0.0)
    got = w.molecule_map[j].float()
    assert torch.allclose(got, ref.float(), rtol=2e-3, atol=2e-3)


def test_genome_pool_collect_layout_matches_sorted_reference():
    """The device collection (pool.hip pool_collect_plan / _move: per-granule sizes and owners, a
    scan, owner copies) lays the pool out exactly as sorting the distinct offsets and summing their
    allocation sizes in that order (plain torch, below), and keeps every genome's bytes."""
    w = _world("cuda", map_size=96, n=1500, s=400)
    g = w._genomes
    for _ in range(3):
        w.divide_cells_t(torch.arange(0, w.n_cells, 3, device="cuda"))
        w.mutate_cells(p=1e-3)
        w.recombinate_cells(p=1e-5)
        w.kill_cells(torch.arange(0, w.n_cells, 5, device="cuda"))
    w._reconcile()
    torch.cuda.synchronize()
    n = g.n
    off, lens = g.off[:n].clone(), g.lens[:n].clone()
    uo, inv = torch.unique(off, return_inverse=True)
    size_u = torch.zeros_like(uo)
    size_u.scatter_reduce_(0, inv, ((lens.to(torch.int64).clamp(min=1) + 15) // 16) * 16, reduce="amax")
    want = (torch.cumsum(size_u, 0) - size_u)[inv]
    before = list(w.cell_genomes)
    g.collect()
    assert torch.equal(g.off[:n], want)
    assert int(g.top.item()) == int(size_u.sum())
    assert list(w.cell_genomes) == before
    g.check()


@pytest.mark.gpu
def test_bench_steps_with_spawns_replay_bit_identically():
    """30 bench steps (chemostat kill / divide, top-up spawns, the genome chains) from the same seed
    in two FRESH worlds -- their initial populations spawned as well -- end bit-identical: the spawn's
    pixel claims are priority rounds (world.hip spawn_claim_coop_kernel: lowest bidder wins, rounds
    behind grid barriers), so a seed fixes which cell gets which pixel (the reference samples free
    pixels from its RNG, world.py:910-920)."""
    import random

    import bench

    atp = CHEMISTRY.molname_2_idx["ATP"]
    runs = []
    for _ in range(2):
        random.seed(21)
        ms.set_seed(21)
        torch.manual_seed(21)
        bench._CHEMOSTAT.update(divided=0, starved=0, steps=0, excess=None, last_d=0, last_s=0)
        w = ms.World(chemistry=CHEMISTRY, map_size=96, device="cuda", seed=21)
        w.spawn_cells(bench.random_genomes(3000, 500, "cuda"))
        spawned = 0
        for _ in range(30):
            st = {}
            bench.step(w, 3000, 500, atp, stats=st)
            spawned += st.get("spawned", 0)
        w.synchronize()
        k = w.kinetics
        runs.append({
            "n": w.n_cells, "spawned": spawned, "positions": w.cell_positions.clone(),
            "molecules": w.cell_molecules.clone(), "lifetimes": w.cell_lifetimes.clone(),
            "divisions": w.cell_divisions.clone(), "cell_map": w.cell_map.clone(), "map": w.molecule_map.clone(),
            "genomes": list(w.cell_genomes), "labels": list(w.cell_labels),
            **{p: getattr(k, p).clone() for p in ("N", "A", "Kmr", "Vmax", "Ke")},
        })
    a, b = runs
    assert a["spawned"] > 0  # (top-ups happened inside the replayed window)
    bad = [key for key in a if not (torch.equal(a[key], b[key]) if isinstance(a[key], torch.Tensor) else a[key] == b[key])]
    assert not bad, bad
    bench._CHEMOSTAT.update(divided=0, starved=0, steps=0, excess=None, last_d=0, last_s=0)


@pytest.mark.gpu
def test_graph_batched_launches_match_direct_launches():
    """With graph batching on, the kernels each native call records go out as one hipGraph launch,
    replayed with updated arguments (csrc/hip/launch.h, opt-in): 20 bench steps (top-ups, chemostat kill / divide, the genome
    chains) from one seed end bit-identical with batching on and with every kernel launched
    directly, and the batched run did launch graphs (and re-used them)."""
    import random

    import bench
    from magicsoup_amd.ops import native

    m = native.hip()
    atp = CHEMISTRY.molname_2_idx["ATP"]
    runs, stats = [], []
    try:
        for on in (False, True):
            m.set_graph_batch(on)
            m.graph_batch_reset()
            random.seed(5)
            ms.set_seed(5)
            torch.manual_seed(5)
            bench._CHEMOSTAT.update(divided=0, starved=0, steps=0, excess=None, last_d=0, last_s=0)
            w = ms.World(chemistry=CHEMISTRY, map_size=96, device="cuda", seed=5)
            w.spawn_cells(bench.random_genomes(3000, 500, "cuda"))
            for _ in range(20):
                bench.step(w, 3000, 500, atp)
            w.synchronize()
            stats.append(m.graph_batch_stats())
            k = w.kinetics
            runs.append({
                "n": w.n_cells, "positions": w.cell_positions.clone(), "molecules": w.cell_molecules.clone(),
                "lifetimes": w.cell_lifetimes.clone(), "divisions": w.cell_divisions.clone(),
                "cell_map": w.cell_map.clone(), "map": w.molecule_map.clone(), "genomes": list(w.cell_genomes),
                **{p: getattr(k, p).clone() for p in ("N", "A", "Kmr", "Vmax", "Ke")},
            })
    finally:
        m.set_graph_batch(False)
        bench._CHEMOSTAT.update(divided=0, starved=0, steps=0, excess=None, last_d=0, last_s=0)
    a, b = runs
    bad = [key for key in a if not (torch.equal(a[key], b[key]) if isinstance(a[key], torch.Tensor) else a[key] == b[key])]
    assert not bad, bad
    assert stats[0]["graph_launches"] == 0
    assert stats[1]["graph_launches"] >= 40 and stats[1]["graph_nodes"] > 2 * stats[1]["graph_launches"], stats[1]
    assert stats[1]["instantiated"] < stats[1]["graph_launches"] // 2, stats[1]  # (replayed, not rebuilt)


def test_gpu_step_loop_is_deterministic():
    """The reference loop as bench.py issues it (activity, kill, lazy division, queued
    recombination + mutation chain, degradation, diffusion next to the chain, lifetimes; no host
    synchronisation besides the API's own) replayed twice from one state with the same seeds ends in
    bit-identical worlds: the device placement, selections, genome chains, speculative activity and
    stencil reductions do not depend on thread timing. (Spawns are covered by
    test_bench_steps_with_spawns_replay_bit_identically.)"""
    import random

    import bench

    atp = CHEMISTRY.molname_2_idx["ATP"]
    base = ms.World(chemistry=CHEMISTRY, map_size=128, device="cuda", seed=3)
    base.spawn_cells(bench.random_genomes(2500, 500, "cuda"))
    base.synchronize()
    runs = []
    for _ in range(2):
        w = copy.deepcopy(base)
        random.seed(9)
        ms.set_seed(9)
        torch.manual_seed(9)
        for _ in range(10):
            w.enzymatic_activity()
            w.kill_cells(w.cell_molecules[:, atp] < 1.0)
            repl = w.cell_molecules[:, atp] > 5.0
            w.cell_molecules[:, atp] -= 4.0 * repl
            w.divide_cells_t(repl, lazy=True)
            w.recombinate_cells(p=1e-5)
            w.mutate_cells(p=1e-4)
            w.degrade_molecules()
            w.diffuse_molecules()
            w.increment_cell_lifetimes()
        w.synchronize()
        k = w.kinetics
        runs.append({
            "n": w.n_cells, "positions": w.cell_positions.clone(), "molecules": w.cell_molecules.clone(),
            "lifetimes": w.cell_lifetimes.clone(), "divisions": w.cell_divisions.clone(),
            "cell_map": w.cell_map.clone(), "map": w.molecule_map.clone(), "genomes": list(w.cell_genomes),
            "labels": list(w.cell_labels), **{p: getattr(k, p).clone() for p in ("N", "A", "Kmr", "Vmax", "Ke")},
        })
    a, b = runs
    assert a["n"] > 500 and int(a["divisions"].sum()) > 0
    bad = [key for key in a if not (torch.equal(a[key], b[key]) if isinstance(a[key], torch.Tensor) else a[key] == b[key])]
    assert not bad, bad


def test_lazy_kill_divide_matches_synchronous_calls():
    """World.kill_divide_t on the GPU (kill, division mask compacted with the survivors, children
    after the device survivor count, no synchronisation) evolves the world bit for bit as
    kill_cells + divide_cells_t(mask[~kill]) do; ops queued meanwhile run against the device state."""
    base = _world("cuda", map_size=64, n=1500, s=400, seed=8)
    base.synchronize()
    atp = CHEMISTRY.molname_2_idx["ATP"]

    def run(fused: bool):
        w = copy.deepcopy(base)
        ms.set_seed(3)
        torch.manual_seed(3)
        sizes = []
        for _ in range(5):
            w.enzymatic_activity()
            a = w.cell_molecules[:, atp]
            kill = a < 1.0
            repl = (a > 3.0) & ~kill
            a -= 2.0 * repl
            if fused:
                w.kill_divide_t(kill, repl)
                assert w.__dict__.get("_count_pending") is not None
            else:
                w.kill_cells(kill)
                w.divide_cells_t(repl[~kill].clone())
            w.recombinate_cells(p=1e-4)
            w.mutate_cells(p=1e-3)
            w.degrade_molecules()
            w.diffuse_molecules()
            assert w.__dict__.get("_count_pending") is None
            w.increment_cell_lifetimes()
            sizes.append(w.n_cells)
        w.synchronize()
        w.check_invariants()
        state = {k: getattr(w, k).clone() for k in ("cell_molecules", "cell_positions", "cell_lifetimes",
                                                     "cell_divisions", "molecule_map", "cell_map")}
        state["Vmax"] = w.kinetics.Vmax.clone()
        return sizes, list(w.cell_genomes), list(w.cell_labels), state

    s0, g0, l0, st0 = run(False)
    s1, g1, l1, st1 = run(True)
    assert s0 == s1 and g0 == g1 and l0 == l1
    for k in st0:
        assert torch.equal(st0[k], st1[k]), k


def test_kill_divide_where_matches_masks_on_gpu():
    """The fused threshold kill / replicate (one native call: masks, payment, kill, division) leaves
    the world bit for bit as the torch masks + kill_divide_t do; a dilution fraction kills about
    that share at random."""
    base = _world("cuda", map_size=64, n=1500, s=400, seed=12)
    base.enzymatic_activity()
    base.synchronize()
    atp = CHEMISTRY.molname_2_idx["ATP"]
    w1, w2 = copy.deepcopy(base), copy.deepcopy(base)
    ms.set_seed(4)
    w1.kill_divide_where(atp, 1.0, 3.0, 2.0)
    ms.set_seed(4)
    a = w2.cell_molecules[:, atp]
    kill = a < 1.0
    div = (a > 3.0) & ~kill
    a -= 2.0 * div
    w2.kill_divide_t(kill, div)
    for k in ("cell_molecules", "cell_positions", "cell_divisions", "cell_lifetimes", "molecule_map", "cell_map"):
        assert torch.equal(getattr(w1, k), getattr(w2, k)), k
    assert list(w1.cell_genomes) == list(w2.cell_genomes) and w1.last_kill == w2.last_kill
    n = w1.n_cells
    w1.kill_divide_where(atp, -1.0, 1e9, kill_fraction=0.3)
    assert 0.6 * n < w1.n_cells < 0.8 * n
    w1.check_invariants()


@pytest.mark.gpu
def test_kill_divide_single_pass_selections_match_two_pass():
    """kill_divide_where with the single-pass selections (survivors + compacted division mask in one
    launch, winners + division commit in one launch: select_lb.h) against the count + write passes
    with the separate mask compaction and commit kernels: the same world, bit for bit."""
    from magicsoup_amd.ops import native

    base = _world("cuda", map_size=96, n=3000, s=400, seed=21)
    base.enzymatic_activity()
    base.synchronize()
    atp = CHEMISTRY.molname_2_idx["ATP"]
    out = []
    try:
        for single in (1, 0):
            native.hip().set_select_single_pass(single)
            w = copy.deepcopy(base)
            ms.set_seed(6)
            for _ in range(3):
                w.kill_divide_where(atp, 1.0, 3.0, 2.0, kill_fraction=0.05)
                w.enzymatic_activity()
            w.synchronize()
            w.check_invariants()
            out.append({k: getattr(w, k).clone() for k in ("cell_molecules", "cell_positions", "cell_divisions",
                                                          "cell_lifetimes", "molecule_map", "cell_map")})
            out[-1]["genomes"] = list(w.cell_genomes)
    finally:
        native.hip().set_select_single_pass(1)
    a, b = out
    assert a["cell_positions"].shape[0] > 1000
    for k in a:
        assert (torch.equal(a[k], b[k]) if isinstance(a[k], torch.Tensor) else a[k] == b[k]), k


def test_kill_divide_with_as_many_kills_as_divisions_refreshes_strings():
    """A kill_divide_t that kills exactly as many cells as it divides leaves n_cells unchanged but
    still compacts the genome / label arenas and appends children: cached string views
    (cell_genomes, cell_labels, read before the call) must show the new rows, as the synchronous
    kill_cells + divide_cells_t do (the count was adopted only when it changed)."""
    base = _world("cuda", map_size=64, n=200, s=300, seed=31)
    base.cell_labels = [f"c{i}" for i in range(base.n_cells)]
    base.synchronize()
    n = base.n_cells
    kill = torch.zeros(n, dtype=torch.bool, device="cuda")
    kill[:10] = True
    div = torch.zeros(n, dtype=torch.bool, device="cuda")
    div[20:30] = True
    ref = copy.deepcopy(base)
    ms.set_seed(2)
    ref.kill_cells(kill)
    ref.divide_cells_t(div[~kill].clone())
    ref.synchronize()
    assert ref.n_cells == n, "the sparse map must place every child (precondition)"
    w = copy.deepcopy(base)
    before_g, before_l = list(w.cell_genomes), list(w.cell_labels)  # (fills the string caches)
    ms.set_seed(2)
    w.kill_divide_t(kill, div)
    w.synchronize()
    assert w.n_cells == n and w.last_kill == (n, n - 10)
    assert list(w.cell_labels) == list(ref.cell_labels) != before_l
    assert list(w.cell_genomes) == list(ref.cell_genomes) != before_g
    assert w.cell_labels[0] == "c10" and w.cell_labels[n - 1] == "c29"
    assert torch.equal(w.cell_positions, ref.cell_positions)


def test_payload_selection_two_pass_matches_single_pass():
    """select_indices_async_pay (the division mask compacted with the survivors) takes the count +
    write passes plus a payload kernel when the single-pass status words do not suffice (> 4M
    cells, forced here with set_select_single_pass(0)): same indices, count and payload bytes."""
    from magicsoup_amd.ops import hip_ops

    m = native.hip()
    g = torch.Generator().manual_seed(5)
    n = 50_000
    src = (torch.rand(n, generator=g) < 0.3).to(torch.uint8).cuda()
    pay = (torch.rand(n, generator=g) < 0.5).to(torch.uint8).cuda()
    out = []
    try:
        for single in (1, 0):
            m.set_select_single_pass(single)
            sel = torch.full((n,), -7, dtype=torch.int64, device="cuda")
            dst = torch.full((n,), 9, dtype=torch.uint8, device="cuda")
            cnt = torch.zeros(2, dtype=torch.int32, device="cuda")
            slot = m.select_indices_async_pay(n, 1, src.data_ptr(), sel.data_ptr(), 0, cnt.data_ptr(), pay.data_ptr(),
                                              dst.data_ptr(), hip_ops._stream())
            torch.cuda.synchronize()
            k = int(m.status_read(slot)[0])
            out.append((k, sel[:k].cpu(), dst.cpu(), int(cnt[0])))
    finally:
        m.set_select_single_pass(1)
    (k1, s1, d1, c1), (k2, s2, d2, c2) = out
    keep = torch.nonzero(src.cpu() == 0).flatten()
    assert k1 == k2 == c1 == c2 == keep.numel()
    assert torch.equal(s1, keep) and torch.equal(s2, keep)
    want = torch.zeros(n, dtype=torch.uint8)
    want[:k1] = pay.cpu()[keep]
    assert torch.equal(d1, want) and torch.equal(d2, want)
    assert not m.lb_error_take()


@pytest.mark.gpu
def test_chain_issued_on_device_count_matches_resolved_count(monkeypatch):
    """A recombinate + mutate pair queued behind a kill_divide is issued before the division's count
    reaches the host (World._chain_bound: sized for 2 n0, the kernels read the device count): the
    same genomes, parameters, molecules and population as issuing it after the count was read."""
    import copy

    from magicsoup_amd.models import world as world_mod

    base = _world("cuda", map_size=96, n=1500, seed=13)
    atp = CHEMISTRY.molname_2_idx["ATP"]
    used = []
    orig = world_mod.World._chain_bound

    def spy(self, q):
        b = orig(self, q)
        used.append(b is not None)
        return b

    monkeypatch.setattr(world_mod.World, "_chain_bound", spy)

    def run(on: bool):
        monkeypatch.setattr(world_mod, "_CHAIN_BOUND", on)
        w = copy.deepcopy(base)
        ms.set_seed(5)
        torch.manual_seed(5)
        for _ in range(6):
            w.enzymatic_activity()
            w.kill_divide_where(atp, kill_below=0.5, divide_above=2.0, divide_cost=1.0)
            w.recombinate_cells(p=2e-5)
            w.mutate_cells(p=2e-4)
            w.degrade_molecules()
            w.diffuse_molecules()
            w.increment_cell_lifetimes()
        w.enzymatic_activity()
        w.synchronize()
        names = ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")
        params = {k: getattr(w.kinetics, k).clone() for k in names}
        from magicsoup_amd.ops import world_ops

        params["_nprot"] = world_ops.translate(w, torch.arange(w.n_cells, device=w.device))[1]
        return w.n_cells, list(w.cell_genomes), params, w.cell_molecules.clone(), w.molecule_map.clone()

    a = run(True)
    assert any(used), "the chain was never issued on the device count"
    used.clear()
    b = run(False)
    assert not any(used)
    assert a[0] == b[0]
    assert a[1] == b[1]
    _assert_params_equal(_real(a[2]), _real(b[2]), a[2]["_nprot"])
    assert torch.equal(a[3], b[3])
    assert torch.equal(a[4], b[4])


@pytest.mark.parametrize("k", [0, 1, 2047, 2048, 5000, 70_000])
def test_place_split_single_pass_matches_two_pass(k):
    """The strip division's winners split by destination (dist.hip place_split): the single-pass
    launch (tile counts published with a generation tag) writes the same parents, pixels, counts and
    headers as the count + write pair, and both match a torch reference of the split."""
    from magicsoup_amd.ops import native

    C, H = 512, 64
    g = torch.Generator().manual_seed(k + 1)
    # placement results: -1 (no pixel) or a pixel of rows 0 .. H + 1 (0 / H + 1: the halo rows)
    px = torch.randint(0, (H + 2) * C, (k,), generator=g)
    px[torch.rand(k, generator=g) < 0.3] = -1
    result = px.cuda()
    cells = torch.randperm(max(k, 1), generator=g)[:k].cuda()
    kk = max(k, 1)
    outs = []
    try:
        for single in (1, 0):
            native.hip().set_split_single(single)
            for use_cells in (True, False):
                par = torch.full((3 * kk,), -7, dtype=torch.int64, device="cuda")
                npos = torch.full((6 * kk,), -7, dtype=torch.int32, device="cuda")
                st = torch.zeros(20, dtype=torch.int32, device="cuda")
                native.hip().place_split(k, result.data_ptr(), cells.data_ptr() if use_cells else 0, C, H,
                                         par.data_ptr(), npos.data_ptr(), st.data_ptr(), st[4:].data_ptr(),
                                         st[8:].data_ptr(), 12, 16, 14, torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                outs.append((single, use_cells, par.cpu(), npos.cpu(), st.cpu()))
    finally:
        native.hip().set_split_single(1)
    x = torch.where(px >= 0, px // C, torch.full_like(px, -1))
    cls = torch.where(px < 0, -1, torch.where(x == 0, 1, torch.where(x == H + 1, 2, 0)))
    for single, use_cells, par, npos, st in outs:
        src = cells.cpu() if use_cells else torch.arange(k)
        for q in range(3):
            sel = torch.nonzero(cls == q).flatten()
            n_q = int(sel.numel())
            assert int(st[q]) == n_q, (single, q)
            assert torch.equal(par[q * kk : q * kk + n_q], src[sel]), (single, use_cells, q)
            pos = npos.view(-1, 2)[q * kk : q * kk + n_q]
            assert torch.equal(pos[:, 0].long(), px[sel] // C) and torch.equal(pos[:, 1].long(), px[sel] % C)
        assert st[4:8].tolist() == [int((cls == 1).sum()), 12, 16, 14]
        assert st[8:12].tolist() == [int((cls == 2).sum()), 12, 16, 14]
    for a, b in zip(outs[:2], outs[2:]):
        assert all(torch.equal(u, v) for u, v in zip(a[2:], b[2:]))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_molecule_totals_match_torch_sums(dtype):
    """World.molecule_totals reads the map once with the pending diffusion correction and
    degradation applied on the fly: equal (to float64 summation order) to torch sums over the
    materialised map and the cell molecules; molecule_means is the reference's logged quantity."""
    w = _world("cuda", map_size=300, n=500)
    if dtype != torch.float32:
        w.__dict__["map_dtype"] = dtype
        w.molecule_map = w.molecule_map.to(dtype)
    w.enzymatic_activity()
    w.degrade_molecules()
    w.diffuse_molecules()
    w.degrade_molecules()  # (a pending scale on top of the pending correction)
    assert w.__dict__.get("_pending_corr") is not None and w.__dict__.get("_pending_scale") is not None
    t = w.molecule_totals().cpu()
    mm = w.molecule_map.double()  # (materialises the pending state)
    want = torch.stack([mm.sum(dim=(1, 2)).cpu(), w.cell_molecules.double().sum(0).cpu()], dim=1)
    # (fp16: the materialisation rounds every corrected value to the storage dtype; the totals are
    # of the fp32 values the readers -- integrator, permeation -- compute with)
    rel = 1e-9 if dtype == torch.float32 else 2e-4
    assert torch.allclose(t, want, rtol=rel, atol=1e-6), (t - want).abs().max()
    means = w.molecule_means()
    ref = [(float(mm[i].sum()) + float(w.cell_molecules[:, i].double().sum())) / (300 * 300 + w.n_cells)
           for i in range(w.n_molecules)]
    assert means == pytest.approx(ref, rel=rel)


def test_ragged_records_match_host_build():
    """Cells built on the GPU take ragged records (csrc/hip/params.h): exactly one per protein of
    their own proteome, none for the padding; their dense view -- records, then the build's padding
    values up to the build width -- equals the host core's dense build of the same genomes."""
    from magicsoup_amd.ops import world_ops

    wc = _world("cpu", map_size=64, n=300, s=500, seed=9)
    wg = _copy_world_cpu_to_gpu(wc)
    rows = torch.arange(wg.n_cells, device="cuda")
    wg._update_params_rows(rows)
    kin = wg.kinetics
    slot = kin.__dict__["_slot"]
    assert slot is not None
    from magicsoup_amd.models.kinetics import _REC_CNT_MASK, _REC_OFF_BITS

    cnt = ((slot >> _REC_OFF_BITS) & _REC_CNT_MASK).cpu()
    _, nprot = world_ops.translate(wc, torch.arange(wc.n_cells))
    assert torch.equal(cnt, nprot.to(torch.int64).cpu())
    # (the copied world's dense rows became records first; a collection keeps only the live runs)
    kin._collect_records(0)
    assert int(kin.__dict__["_rtop"].item()) == int(nprot.sum())
    assert torch.equal(((kin.__dict__["_slot"] >> _REC_OFF_BITS) & _REC_CNT_MASK).cpu(), cnt)
    P = wc.kinetics.N.size(1)
    for name in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke"):
        a, b = getattr(kin, name)[:, :P].cpu(), getattr(wc.kinetics, name)
        if a.dtype == torch.int32:
            assert torch.equal(a, b), name
        else:
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-30, equal_nan=True), name
    # the same activity from the records and from the dense layout they materialise to
    wd = copy.deepcopy(wg)  # (the copy holds the dense tensors read above)
    assert wd.kinetics.__dict__["_slot"] is None
    wg2 = copy.deepcopy(wg)
    wg2._update_params_rows(rows)  # records again
    for w in (wd, wg2):
        w.enzymatic_activity()
    assert torch.equal(wd.cell_molecules, wg2.cell_molecules)
