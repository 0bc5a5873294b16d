"""Kinetics: parameter derivation and the integrator (reference tests/fast/test_kinetics.py).

Both native paths (host core here, HIP kernel in tests/test_gpu_kernels.py) are checked against a
plain float64 loop transcription of the reference semantics (kinetics.py:521-625 parameter build,
771-918 velocities / negative guard / equilibrium damping), plus closed-form and property checks."""
import math

import numpy as np
import pytest
import torch

import magicsoup_amd as ms
from magicsoup_amd.constants import EPS, GAS_CONSTANT, MAX, MIN
from magicsoup_amd.models.kinetics import Kinetics
from magicsoup_amd.ops import kinetics_ops

_MA = ms.Molecule("KTa", energy=15e3)
_MB = ms.Molecule("KTb", energy=10e3)
_MC = ms.Molecule("KTc", energy=10e3)
_MD = ms.Molecule("KTd", energy=5e3)
_CHEM = ms.Chemistry(
    molecules=[_MA, _MB, _MC, _MD],
    reactions=[([_MA], [_MB]), ([_MB], [_MC]), ([_MB, _MC], [_MD]), ([_MD], [_MB, _MB])],
)


# --------------------------------------------------------------------------------------------- oracle
def _nanmean(vals):
    v = [x for x in vals if not math.isnan(x)]
    return sum(v) / len(v) if v else 0.0


def _oracle_params(kin: Kinetics, proteome, P: int):
    """Per-protein parameters of one proteome, float64 loops over the reference's definitions."""
    vmax_w = kin.vmax_map.weights.double().tolist()
    km_w = kin.km_map.weights.double().tolist()
    signs = kin.sign_map.signs.tolist()
    hills = kin.hill_map.numbers.tolist()
    RM, TM, EM = kin.reaction_map.M.tolist(), kin.transport_map.M.tolist(), kin.effector_map.M.tolist()
    E = kin.mol_energies.double().tolist()
    s = len(E)
    out = {k: [] for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")}
    for p in range(P):
        doms = proteome[p][0] if p < len(proteome) else []
        N = [0] * s
        Nf = [0] * s
        Nb = [0] * s
        A = [0] * s
        kmr_lists = [[] for _ in range(s)]
        vmaxs, kmns = [], []
        for (t, i0, i1, i2, i3), *_ in doms:
            sign, km = signs[i2], km_w[i1]
            if t == 3:
                vec = EM[i3]
                for j in range(s):
                    A[j] += vec[j] * sign * hills[i0]
                    if vec[j] != 0 and not math.isnan(km):
                        kmr_lists[j].append(vec[j] * km)
                continue
            vmaxs.append(vmax_w[i0])
            kmns.append(km)
            vec = RM[i3] if t == 1 else TM[i3]
            for j in range(s):
                nd = vec[j] * sign
                N[j] += nd
                Nf[j] += max(-nd, 0)
                Nb[j] += max(nd, 0)
        kmr = [(_nanmean(k) if k else 0.0) ** a if (k or a == 0) else (0.0 if a > 0 else math.inf) for k, a in
               zip(kmr_lists, A)]
        kmn = _nanmean(kmns)
        e = sum(n * ej for n, ej in zip(N, E))
        ke = min(max(math.exp(-e / kin.abs_temp / GAS_CONSTANT), EPS), MAX)
        kmf = kmn if ke >= 1 else kmn / ke
        kmb = kmn * ke if ke >= 1 else kmn
        out["N"].append(N)
        out["Nf"].append(Nf)
        out["Nb"].append(Nb)
        out["A"].append(A)
        out["Kmr"].append(kmr)
        out["Vmax"].append(_nanmean(vmaxs))
        out["Ke"].append(ke)
        out["Kmf"].append(min(max(kmf, EPS), MAX))
        out["Kmb"].append(min(max(kmb, EPS), MAX))
    return {k: np.array(v, dtype=np.float64) for k, v in out.items()}


def _prod_pow(x, n):
    """prod_j x_j^n_j over n_j > 0; (value, involved) like the reference's _multiply_signals."""
    involved = any(v > 0 for v in n)
    if not involved:
        return 0.0, False
    r = 1.0
    for xj, nj in zip(x, n):
        if nj > 0:
            r *= xj**nj
    if math.isnan(r) or r < 0:
        r = 0.0
    return min(r, MAX), True


def _velocity_part(p, X0, trim):
    """Velocities, negative-guarded NV and the undamped candidate of one part for one cell (float64)."""
    P, s = p["N"].shape
    V = np.zeros(P)
    for k in range(P):
        kf, f_inv = _prod_pow(X0, p["Nf"][k])
        kb, b_inv = _prod_pow(X0, p["Nb"][k])
        kf = min(kf / p["Kmf"][k], MAX) if f_inv else 0.0
        kb = min(kb / p["Kmb"][k], MAX) if b_inv else 0.0
        acat = (kf - kb) / (1 + kf + kb)
        areg = 1.0
        for j in range(s):
            a = p["A"][k][j]
            if a == 0:
                continue
            with np.errstate(divide="ignore", invalid="ignore"):
                xa = np.float64(X0[j]) ** a if X0[j] != 0 or a > 0 else math.inf
                r = xa / (xa + p["Kmr"][k][j])
            areg *= 1.0 if math.isnan(r) else r
        areg = min(areg, MAX)
        V[k] = min(max(acat * max(p["Vmax"][k] * trim, 0.0) * areg, MIN), MAX)
    NV = p["N"] * V[:, None]
    cons = np.clip(-NV, 0, None).sum(0)
    with np.errstate(divide="ignore", invalid="ignore"):
        F = np.minimum(X0 / cons, 1.0)
    fmin = np.ones(P)
    for k in range(P):
        for j in range(s):
            if NV[k, j] < 0:
                fmin[k] = min(fmin[k], F[j]) if not math.isnan(F[j]) else math.nan
    NV = NV * fmin[:, None]
    return V, NV, np.maximum(X0 + NV.sum(0), 0.0)


def _qke(p, X1):
    P = p["N"].shape[0]
    q = np.zeros(P)
    for k in range(P):
        pb, bi = _prod_pow(X1, p["Nb"][k])
        ps, si = _prod_pow(X1, p["Nf"][k])
        with np.errstate(divide="ignore", invalid="ignore"):
            qq = np.float64(pb if bi else 0.0) / np.float64(ps if si else 0.0)
        q[k] = 1.0 if math.isnan(qq) else min(max(qq, EPS), MAX)
    return q / p["Ke"]


def _oracle_population(params, X, trims, n_iters, exits=None, margin=1e-4, decisions=None, report=None):
    """The reference's integration over a whole population (float64): per part, velocities and the
    negative guard per cell, then the equilibrium damping whose early exit is the population-wide
    ``torch.any`` (kinetics.py:846). ``exits`` (per part: damping iterations that ran, from the
    native core's flags) replays the native exit decisions instead of deciding in float64.

    ``decisions`` (uint8 (c, parts, 4, P) from the native host core): replay the native per-protein
    damping decisions instead of deciding in float64; ``report`` (list) then receives
    (cell, part, iteration, protein, ill_conditioned) for every decision where the two disagree.

    Returns (X, borderline): ``borderline[c]`` is True if one of the cell's damping decisions had
    Q/Ke within a relative ``margin`` of a threshold (1.5, 1/1.5), or involved a species the step
    nearly exhausted (X1 within 1e-4 of 0 relative to X0: the difference of two nearly equal
    numbers) -- such a decision can go either way between float32 and float64 and is not a
    meaningful disagreement."""
    X = [np.array(x, dtype=np.float64) for x in X]
    border = [False] * len(X)
    for part, trim in enumerate(trims):
        parts = [_velocity_part(p, x, trim) for p, x in zip(params, X)]
        X0 = X
        X1 = [c[2] for c in parts]
        if n_iters:
            Fa = [np.ones(p["N"].shape[0]) for p in params]
            for it, inc in enumerate((0.5, 0.25, 0.125, 0.0625)[:n_iters]):
                lows, highs, anyflag = [], [], False
                for c, p in enumerate(params):
                    V, NV, _ = parts[c]
                    qke = _qke(p, X1[c])
                    imp, fwd = np.abs(V) > 0.1, V > 0
                    near = (np.abs(qke * 1.5 - 1.0) < margin) | (np.abs(qke / 1.5 - 1.0) < margin)
                    # a velocity at the noise level of its Vmax: its sign (the reaction direction
                    # the damping reads) is not determined by float32 vs float64
                    with np.errstate(invalid="ignore"):
                        near |= np.abs(V) < 1e-4 * np.abs(p["Vmax"] * trim)
                    low = np.where(fwd, qke < 1 / 1.5, qke > 1.5) & ~(fwd & (Fa[c] == 1.0))
                    high = np.where(fwd, qke > 1.5, qke < 1 / 1.5) & ~(~fwd & (Fa[c] == 0.0))
                    # a species the step (nearly) exhausted: X1 = X0 - consumption cancels, so its
                    # float32 value is only known to ~1e-6 of X0; a decision that changes when such a
                    # species moves by that much is ill-conditioned
                    drained = X1[c] < 1e-4 * np.maximum(X0[c], 1.0)
                    if drained.any():
                        # (the float32 residual of the cancellation can be anything below ~1e-6 X0)
                        trials = [np.where(drained, 0.0, X1[c])]
                        for j in np.nonzero(drained)[0]:
                            z = X1[c].copy()
                            z[j] = 0.0
                            trials.append(z)
                        for rel in (1e-6, 1e-8, 1e-10, 1e-12):
                            d = np.where(drained, rel * np.maximum(X0[c], 1.0), 0.0)
                            trials += [X1[c] + d, np.maximum(X1[c] - d, 0.0)]
                            for j in np.nonzero(drained)[0]:  # each drained species on its own
                                e = np.zeros_like(d)
                                e[j] = d[j]
                                trials += [X1[c] + e, np.maximum(X1[c] - e, 0.0)]
                        for xp in trials:
                            qp = _qke(p, xp)
                            lp = np.where(fwd, qp < 1 / 1.5, qp > 1.5) & ~(fwd & (Fa[c] == 1.0))
                            hp = np.where(fwd, qp > 1.5, qp < 1 / 1.5) & ~(~fwd & (Fa[c] == 0.0))
                            near |= (lp != low) | (hp != high)
                    if (near & (NV != 0).any(axis=1)).any():
                        border[c] = True
                    if decisions is not None:
                        d = decisions[c, part, it, : len(low)]
                        nl, nh = (d & 1) != 0, (d & 2) != 0
                        for k in np.nonzero((nl != low) | (nh != high))[0]:
                            if report is not None:
                                report.append((c, part, it, int(k), bool(near[k])))
                        low, high = nl, nh
                    lows.append(low)
                    highs.append(high)
                    anyflag |= bool(((low | high) & imp).any())
                stop = (it >= exits[part]) if exits is not None else not anyflag
                if stop:
                    break
                for c, p in enumerate(params):
                    Fa[c] = np.clip(Fa[c] - inc * highs[c] + inc * lows[c], 0, 1)
                    X1[c] = np.maximum(X0[c] + (parts[c][1] * Fa[c][:, None]).sum(0), 0.0)
        X = X1
    return X, border


def _exits(masks, n_iters):
    """Damping iterations each part ran, from the native per-part flag bits (bit i: iteration i
    still had an impactful correction somewhere)."""
    out = []
    for bits in masks:
        k = 0
        while k < n_iters and (bits >> k) & 1:
            k += 1
        out.append(k)
    return out


# --------------------------------------------------------------------------------------------- helpers
def _kinetics(seed=0) -> Kinetics:
    import random

    random.seed(seed)
    g = ms.Genetics()
    kin = Kinetics(chemistry=_CHEM, scalar_enc_size=max(g.one_codon_map.values()),
                   vector_enc_size=max(g.two_codon_map.values()))
    return kin, g


def _setup(n_cells=40, seed=0, size=900):
    kin, g = _kinetics(seed)
    rng = np.random.default_rng(seed)
    genomes = ["".join(rng.choice(list("TCGA"), size=size)) for _ in range(n_cells)]
    proteomes = g.translate_genomes(genomes)
    kin.increase_max_cells(n_cells)
    kin.increase_max_proteins(max(1, max(len(p) for p in proteomes)))
    kin.set_cell_params(list(range(n_cells)), proteomes)
    return kin, proteomes


# --------------------------------------------------------------------------------------------- params
def test_params_match_reference_definitions():
    kin, proteomes = _setup()
    P = kin.N.size(1)
    for c, prot in enumerate(proteomes):
        exp = _oracle_params(kin, prot, P)
        for k in ("N", "Nf", "Nb", "A"):
            assert np.array_equal(getattr(kin, k)[c].numpy(), exp[k].astype(np.int64)), (c, k)
        for k in ("Vmax", "Ke", "Kmf", "Kmb"):
            assert np.allclose(getattr(kin, k)[c].double().numpy(), exp[k], rtol=1e-4, atol=0), (c, k)
        got = kin.Kmr[c].double().numpy()
        fin = np.isfinite(exp["Kmr"])
        assert np.allclose(got[fin], exp["Kmr"][fin], rtol=1e-4), c


def test_hand_built_transporter_and_catalytic_protein():
    kin, _ = _kinetics()
    m = len(_CHEM.molecules)
    # token maps chosen by hand: vmax idx 1 -> 2.0, km idx 1 -> 0.5, idx 2 -> 1.5
    kin.vmax_map.weights = torch.tensor([math.nan, 2.0, 4.0])
    kin.km_map.weights = torch.tensor([math.nan, 0.5, 1.5])
    kin.sign_map.signs = torch.tensor([0, 1, -1], dtype=torch.int32)
    kin.hill_map.numbers = torch.tensor([0, 1, 3], dtype=torch.int32)
    RM = torch.zeros(3, 2 * m, dtype=torch.int32)
    RM[1, [0, 1]] = torch.tensor([-1, 1], dtype=torch.int32)  # a -> b
    TM = torch.zeros(3, 2 * m, dtype=torch.int32)
    TM[1, [1, m + 1]] = torch.tensor([-1, 1], dtype=torch.int32)  # b in -> b out
    EM = torch.zeros(3, 2 * m, dtype=torch.int32)
    EM[1, 3] = 1  # effector d (inside)
    kin.reaction_map.M, kin.transport_map.M, kin.effector_map.M = RM, TM, EM
    prot = [
        ([((1, 1, 1, 1, 1), 0, 21), ((2, 2, 2, 2, 1), 21, 42), ((3, 2, 2, 1, 1), 42, 63)], 0, 63, True),
    ]
    kin.increase_max_cells(1)
    kin.increase_max_proteins(2)
    kin.set_cell_params([0], [prot])
    # catalytic a->b fwd, transporter b in->out reversed: N = -a + b - (-b_in + b_out)
    exp_N = [0] * (2 * m)
    exp_N[0], exp_N[1], exp_N[m + 1] = -1, 2, -1
    assert kin.N[0, 0].tolist() == exp_N
    assert kin.Nf[0, 0].tolist() == [1, 0, 0, 0, 0, 1, 0, 0]
    assert kin.Nb[0, 0].tolist() == [0, 2, 0, 0, 0, 0, 0, 0]
    assert kin.Vmax[0, 0].item() == pytest.approx(3.0)  # mean(2.0, 4.0); regulatory excluded
    assert kin.A[0, 0].tolist() == [0, 0, 0, 3, 0, 0, 0, 0]  # sign +1 * hill 3
    assert kin.Kmr[0, 0, 3].item() == pytest.approx(1.5**3, rel=1e-5)
    e = -_MA.energy + 2 * _MB.energy - _MB.energy  # b outside has b's energy
    ke = math.exp(-e / 310.0 / GAS_CONSTANT)
    assert kin.Ke[0, 0].item() == pytest.approx(ke, rel=1e-4)
    kmn = (0.5 + 1.5) / 2
    kmf, kmb = (kmn, kmn * ke) if ke >= 1 else (kmn / ke, kmn)
    assert kin.Kmf[0, 0].item() == pytest.approx(kmf, rel=1e-4)
    assert kin.Kmb[0, 0].item() == pytest.approx(kmb, rel=1e-4)
    # padding protein slot: Ke 1, Km EPS, everything else 0
    assert kin.Vmax[0, 1].item() == 0 and kin.Ke[0, 1].item() == 1.0
    assert (kin.N[0, 1] == 0).all()
    # human readable view
    views = kin.get_proteome(prot)
    assert len(views) == 1 and len(views[0].domains) == 3
    assert isinstance(views[0].domains[0], ms.CatalyticDomain)
    assert views[0].domains[0].substrates == [_MA] and views[0].domains[0].products == [_MB]
    assert isinstance(views[0].domains[1], ms.TransporterDomain) and views[0].domains[1].molecule is _MB
    assert isinstance(views[0].domains[2], ms.RegulatoryDomain) and views[0].domains[2].effector is _MD


def test_unset_copy_remove_and_grow():
    kin, proteomes = _setup(n_cells=10)
    N = kin.N.clone()
    Vmax = kin.Vmax.clone()
    kin.copy_cell_params(from_idxs=[0, 1], to_idxs=[8, 9])
    assert torch.equal(kin.N[8:], N[:2]) and torch.equal(kin.Vmax[8:], Vmax[:2])
    kin.unset_cell_params([3])
    assert (kin.N[3] == 0).all() and (kin.Vmax[3] == 0).all()
    keep = torch.tensor([True] * 5 + [False] * 5)
    kin.remove_cell_params(keep=keep)
    assert kin.N.size(0) == 5 and torch.equal(kin.N[:3], N[:3])
    kin.increase_max_cells(by_n=4)
    assert kin.N.size(0) == 9 and (kin.N[5:] == 0).all()
    p0 = kin.N.size(1)
    kin.increase_max_proteins(p0 + 3)
    assert kin.N.size(1) == p0 + 3 and (kin.N[:, p0:] == 0).all()
    assert torch.equal(kin.N[:3, :p0], N[:3])


def test_params_written_into_assigned_tensors():
    """Assigning parameter tensors then setting params writes into those tensors (reference
    tests assign zeros and read them back)."""
    kin, g = _kinetics()
    s = kin.n_signals
    N = torch.zeros(2, 3, s, dtype=torch.int32)
    Vmax = torch.zeros(2, 3)
    kin.N, kin.Vmax = N, Vmax
    for name in ("Nf", "Nb", "A"):
        setattr(kin, name, torch.zeros(2, 3, s, dtype=torch.int32))
    kin.Kmr = torch.zeros(2, 3, s)
    for name in ("Kmf", "Kmb", "Ke"):
        setattr(kin, name, torch.zeros(2, 3))
    prots = g.translate_genomes([ms.random_genome(2000) for _ in range(30)])
    prots = [p[:3] for p in prots if len(p) >= 1][:2]
    kin.set_cell_params([0, 1], prots)
    assert kin.N is N and kin.Vmax is Vmax
    assert (N != 0).any() and (Vmax > 0).any()


# --------------------------------------------------------------------------------------------- integrator
def _params_np(kin, c):
    return {k: getattr(kin, k)[c].double().numpy() for k in ("N", "Nf", "Nb", "A", "Kmr", "Kmf", "Kmb", "Vmax", "Ke")}


@pytest.mark.parametrize("n_iters", [0, 4])
def test_integrator_matches_float64_oracle(n_iters):
    """Native integrator vs the float64 population oracle, decision-aware: the oracle replays the
    native core's population-wide exit decisions, and cells with a damping decision within 1e-4 of
    a Q/Ke threshold (which float32 vs float64 rounding may flip) are set aside -- few of them,
    and every other cell must agree."""
    kin, _ = _setup(n_cells=60, seed=1)
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.gamma(2.0, 2.0, size=(60, kin.n_signals)).astype(np.float32))
    _decision_aware_check(kin, X, n_iters)


def test_integrator_matches_float64_oracle_on_a_world_population():
    """A Wood-Ljungdahl world (400 random 500 bp genomes, its own map pixels): many cells exhaust a
    species within a step, which makes the damping decisions hinge on float rounding; replaying the
    native decisions, the trajectories agree for every cell."""
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY
    from tests.conftest import gen_genomes

    ms.set_seed(1)
    torch.manual_seed(1)
    w = ms.World(chemistry=CHEMISTRY, map_size=64, seed=1)
    w.spawn_cells(gen_genomes(400, 500))
    pos = w.cell_positions.long()
    X = torch.cat([w.cell_molecules, w.molecule_map[:, pos[:, 0], pos[:, 1]].T], dim=1).contiguous()
    close, report = _decision_aware_check(w.kinetics, X, 4)
    assert close.all()


def _decision_aware_check(kin, X, n_iters):
    """The native host core against the float64 population oracle replaying the native exit and
    per-protein damping decisions: every cell must agree (>= 0.999), and every decision where
    float64 would have decided otherwise must be ill-conditioned (Q/Ke at a threshold, or hinging
    on a species the step nearly exhausted)."""
    c = X.size(0)
    P = kin.N.size(1)
    Xk = X.clone()
    dec = np.zeros((c, 3, 4, P), dtype=np.uint8)
    masks = kinetics_ops.integrate(kin, Xk, trims=(0.7, 0.2, 0.1), n_iters=n_iters, decisions=dec)
    params = [_params_np(kin, i) for i in range(c)]
    exits = _exits(masks, n_iters) if n_iters else None
    report = []
    ref, border = _oracle_population(params, X.double().numpy(), (0.7, 0.2, 0.1), n_iters, exits=exits,
                                     decisions=dec if n_iters else None, report=report)
    close = np.array([np.allclose(Xk[i].double().numpy(), ref[i], rtol=2e-3, atol=2e-3) for i in range(c)])
    assert close.mean() >= 0.999, (close.mean(), np.nonzero(~close))
    bad = [r for r in report if not r[4]]
    assert not bad, bad[:10]
    return close, report


def test_empty_cells_are_unchanged_and_outputs_non_negative():
    kin, _ = _setup(n_cells=30, seed=2)
    kin.unset_cell_params(list(range(0, 30, 3)))
    X = torch.rand(30, kin.n_signals) * 5
    X[::5] = 0.0
    Y = kin.integrate_signals(X)
    assert torch.equal(Y[::3], X[::3])
    assert (Y >= 0).all() and torch.isfinite(Y).all()
    assert not torch.equal(Y, X)


def test_simple_reaction_conserves_and_approaches_equilibrium():
    kin, _ = _kinetics()
    m = len(_CHEM.molecules)
    kin.vmax_map.weights = torch.tensor([math.nan, 5.0])
    kin.km_map.weights = torch.tensor([math.nan, 1.0])
    kin.sign_map.signs = torch.tensor([0, 1], dtype=torch.int32)
    RM = torch.zeros(2, 2 * m, dtype=torch.int32)
    RM[1, [0, 1]] = torch.tensor([-1, 1], dtype=torch.int32)  # a -> b, releases 5 kJ: Ke = exp(5000 / (R T)) ~ 7
    kin.reaction_map.M = RM
    kin.increase_max_cells(1)
    kin.increase_max_proteins(1)
    kin.set_cell_params([0], [[([((1, 1, 1, 1, 1), 0, 21)], 0, 21, True)]])
    ke = kin.Ke[0, 0].item()
    assert ke == pytest.approx(math.exp(5e3 / 310 / GAS_CONSTANT), rel=1e-4)
    X = torch.zeros(1, 2 * m)
    X[0, 0] = 10.0  # only substrate: a zero product must not stop the reaction
    for _ in range(30):
        X = kin.integrate_signals(X)
        assert X[0, 0] + X[0, 1] == pytest.approx(10.0, rel=1e-5)
    assert X[0, 1] / X[0, 0] == pytest.approx(ke, rel=0.2)


def test_negative_concentrations_are_prevented():
    kin, _ = _kinetics()
    m = len(_CHEM.molecules)
    kin.vmax_map.weights = torch.tensor([math.nan, 100.0])
    kin.km_map.weights = torch.tensor([math.nan, 0.01])
    kin.sign_map.signs = torch.tensor([0, 1], dtype=torch.int32)
    RM = torch.zeros(3, 2 * m, dtype=torch.int32)
    RM[1, [0, 1]] = torch.tensor([-1, 1], dtype=torch.int32)  # a -> b
    RM[2, [0, 2]] = torch.tensor([-1, 1], dtype=torch.int32)  # a -> c
    kin.reaction_map.M = RM
    kin.increase_max_cells(1)
    kin.increase_max_proteins(2)
    prots = [([((1, 1, 1, 1, 1), 0, 21)], 0, 21, True), ([((1, 1, 1, 1, 2), 0, 21)], 0, 21, True)]
    kin.set_cell_params([0], [prots])
    X = torch.zeros(1, 2 * m)
    X[0, 0] = 1.0
    Y = kin.integrate_signals(X)
    assert (Y >= 0).all()
    assert Y[0, :3].sum() == pytest.approx(1.0, rel=1e-5)
    assert Y[0, 1] == pytest.approx(Y[0, 2].item(), rel=1e-4)  # both drain a equally


def test_inhibitor_slows_reaction():
    kin, _ = _kinetics()
    m = len(_CHEM.molecules)
    kin.vmax_map.weights = torch.tensor([math.nan, 1.0])
    kin.km_map.weights = torch.tensor([math.nan, 1.0])
    kin.sign_map.signs = torch.tensor([0, 1, -1], dtype=torch.int32)
    kin.hill_map.numbers = torch.tensor([0, 2], dtype=torch.int32)
    RM = torch.zeros(2, 2 * m, dtype=torch.int32)
    RM[1, [0, 1]] = torch.tensor([-1, 1], dtype=torch.int32)
    EM = torch.zeros(2, 2 * m, dtype=torch.int32)
    EM[1, 3] = 1
    kin.reaction_map.M, kin.effector_map.M = RM, EM
    kin.increase_max_cells(2)
    kin.increase_max_proteins(1)
    plain = [([((1, 1, 1, 1, 1), 0, 21)], 0, 42, True)]
    inhib = [([((1, 1, 1, 1, 1), 0, 21), ((3, 1, 1, 2, 1), 21, 42)], 0, 42, True)]
    kin.set_cell_params([0, 1], [plain, inhib])
    assert kin.A[1, 0, 3].item() == -2
    X = torch.zeros(2, 2 * m)
    X[:, 0] = 2.0
    X[:, 3] = 3.0
    Y = kin.integrate_signals(X)
    made_plain, made_inhib = Y[0, 1].item(), Y[1, 1].item()
    assert 0 < made_inhib < made_plain
    # inhibitor absent (X=0) -> full activity
    X[1, 3] = 0.0
    Y = kin.integrate_signals(X)
    assert Y[1, 1].item() == pytest.approx(made_plain, rel=1e-5)


def test_torch_stage_oracle_agrees_with_native():
    """The reference-shaped torch stages kept on Kinetics (used when a subclass overrides them)
    reproduce the native fused integrator."""
    kin, _ = _setup(n_cells=40, seed=5)
    X = torch.rand(40, kin.n_signals) * 4
    Y = kin.integrate_signals(X)

    class Staged(Kinetics):
        def _multiply_signals(self, X, N):  # force the torch path
            return Kinetics._multiply_signals(self, X, N)

    kin.__class__ = Staged
    Z = kin.integrate_signals(X)
    kin.__class__ = Kinetics
    close = torch.isclose(Y, Z, rtol=1e-3, atol=1e-3).all(dim=1).numpy()
    # both are float32 with different operation orders: only cells with a damping decision at a
    # Q/Ke threshold (float64 oracle, relative margin 1e-3) may differ
    params = [_params_np(kin, c) for c in range(40)]
    _, border = _oracle_population(params, X.double().numpy(), (0.7, 0.2, 0.1), 4, margin=1e-3)
    border = np.array(border)
    # (a cell counts as ill-conditioned when any of its decisions is: the bulk still agrees outright)
    assert close.mean() >= 0.95 and close[~border].all(), (close.mean(), np.nonzero(~close & ~border))
