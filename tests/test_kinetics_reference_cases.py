"""Parameter building and kinetics helpers pinned to the reference's own hand-computed values.

The deterministic token maps (Km / Vmax weights, signs, Hill numbers, transporter / effector /
reaction vectors) and the expected values of the reference's fixture tests are reproduced here:

* transporter / regulatory / catalytic parameter building:
  ``tests/fast/test_kinetics.py:122-953`` (``test_cell_params_with_*_domains``);
* ``_multiply_signals`` / ``_get_quotient`` edge cases with ``_MAX`` / ``_EPS``:
  ``tests/fast/test_kinetics.py:1697-1853``.

Each parameter case is checked on the host core's parameter build and, on a GPU box, on the HIP
``build_params`` kernel. The expected tables are the reference's assertions (dense per-protein
rows where the reference asserts "all other entries are 0").
"""
import math

import pytest
import torch

import magicsoup_amd as ms
from magicsoup_amd.constants import EPS, GAS_CONSTANT, MAX
from magicsoup_amd.models.kinetics import Kinetics

_TOL = 1e-4
_a = ms.Molecule("RefKa", energy=15e3)
_b = ms.Molecule("RefKb", energy=10e3)
_c = ms.Molecule("RefKc", energy=10e3)
_d = ms.Molecule("RefKd", energy=5e3)
_CHEM = ms.Chemistry(molecules=[_a, _b, _c, _d],
                     reactions=[([_a], [_b]), ([_b], [_c]), ([_b, _c], [_d]), ([_d], [_b, _b])])


def _vec(*pairs, n=8):
    v = [0] * n
    for i, x in pairs:
        v[i] = x
    return v


# token -> value maps of the reference fixtures (idx 0 = "empty")
_KM = [math.nan] + [0.1 * i for i in range(1, 30)]
_VMAX = [math.nan] + [1.0 + 0.1 * i for i in range(1, 20)]
_SIGNS = [0, 1, -1]
_HILLS = [0, 1, 2, 3, 4, 5]
_TRANSPORT = [_vec()] + [_vec((k, -1), (k + 4, 1)) for k in range(4)] + [_vec()] * 4
_EFFECTOR = [_vec()] + [_vec((k, 1)) for k in range(8)]
_REACTION = [_vec(), _vec((0, -1), (1, 1)), _vec((1, -1), (2, 1)), _vec((1, -1), (2, -1), (3, 1)),
             _vec((1, 2), (3, -1))] + [_vec()] * 4


def _kinetics(device="cpu") -> Kinetics:
    g = ms.Genetics()
    kin = Kinetics(chemistry=_CHEM, abs_temp=310, device=device, scalar_enc_size=max(g.one_codon_map.values()),
                   vector_enc_size=max(g.two_codon_map.values()))
    kin.km_map.weights = torch.tensor(_KM, dtype=torch.float32, device=device)
    kin.vmax_map.weights = torch.tensor(_VMAX, dtype=torch.float32, device=device)
    kin.sign_map.signs = torch.tensor(_SIGNS, dtype=torch.int32, device=device)
    kin.hill_map.numbers = torch.tensor(_HILLS, dtype=torch.int32, device=device)
    kin.transport_map.M = torch.tensor(_TRANSPORT, dtype=torch.int32, device=device)
    kin.effector_map.M = torch.tensor(_EFFECTOR, dtype=torch.int32, device=device)
    kin.reaction_map.M = torch.tensor(_REACTION, dtype=torch.int32, device=device)
    return kin


def _ke(subs, prods):
    e = sum(m.energy for m in prods) - sum(m.energy for m in subs)
    return math.exp(-e / 310 / GAS_CONSTANT)


def _mean(*x):
    return sum(x) / len(x)


def _prot(doms, start, end, fwd):
    """Reference proteome spec: domains ((type, i0, i1, i2, i3), start, end)."""
    return ([(tuple(spec), s, e) for spec, s, e in doms], start, end, fwd)


# ------------------------------------------------------------------------------------ cases
# Each case: two cells' proteomes and, per (cell, protein), the expected parameters. Scalars
# Ke / Kmf / Kmb / Vmax; N / Nf / Nb / A as dense signal rows; Kmr as {signal: value} (other signals
# are not regulated: Kmr <= 1 as the reference asserts).
_KE_AB = _ke([_a], [_b])

TRANSPORTER = dict(
    cells=[
        [_prot([((2, 5, 5, 1, 1), 6, 27)], 13, 27, True),
         _prot([((2, 5, 5, 1, 1), 5, 13), ((2, 1, 2, 2, 1), 7, 12)], 36, 74, False)],
        [_prot([((2, 5, 4, 1, 1), 1, 10), ((2, 4, 5, 1, 1), 2, 20), ((2, 3, 6, 1, 2), 3, 30),
                ((2, 2, 7, 1, 3), 4, 40)], 91, 112, False),
         _prot([((1, 10, 5, 1, 1), 5, 50), ((2, 5, 5, 1, 1), 6, 60)], 1, 10, False)],
    ],
    expect={
        (0, 0): dict(Ke=1.0, Kmf=0.5, Kmb=0.5, Vmax=1.5, N=_vec((0, -1), (4, 1)), Nf=_vec((0, 1)),
                     Nb=_vec((4, 1))),
        (0, 1): dict(Ke=1.0, Kmf=_mean(0.5, 0.2), Kmb=_mean(0.5, 0.2), Vmax=_mean(1.5, 1.1), N=_vec(),
                     Nf=_vec((0, 1), (4, 1)), Nb=_vec((0, 1), (4, 1))),
        (0, 2): dict(Kmf=0.0, Kmb=0.0, Vmax=0.0, N=_vec(), Nf=_vec(), Nb=_vec()),
        (1, 0): dict(Ke=1.0, Kmf=_mean(0.4, 0.5, 0.6, 0.7), Kmb=_mean(0.4, 0.5, 0.6, 0.7),
                     Vmax=_mean(1.5, 1.4, 1.3, 1.2), N=_vec((0, -2), (1, -1), (2, -1), (4, 2), (5, 1), (6, 1)),
                     Nf=_vec((0, 2), (1, 1), (2, 1)), Nb=_vec((4, 2), (5, 1), (6, 1))),
        (1, 1): dict(Ke=_KE_AB, Kmf=0.5, Kmb=0.5 * _KE_AB, Vmax=_mean(2.0, 1.5), N=_vec((0, -2), (1, 1), (4, 1)),
                     Nf=_vec((0, 2)), Nb=_vec((1, 1), (4, 1))),
        (1, 2): dict(Kmf=0.0, Kmb=0.0, Vmax=0.0, N=_vec(), Nf=_vec(), Nb=_vec()),
    },
    A_zero=True,
)

REGULATORY = dict(
    cells=[
        [_prot([((1, 10, 5, 1, 1), 1, 10), ((3, 1, 10, 1, 3), 2, 20), ((3, 2, 20, 2, 4), 3, 30)], 1, 100, False),
         _prot([((1, 10, 5, 1, 1), 4, 40), ((3, 1, 10, 1, 1), 5, 50), ((3, 3, 15, 1, 5), 6, 60)], 2, 200, True)],
        [_prot([((1, 10, 5, 1, 1), 7, 70), ((3, 1, 10, 2, 2), 8, 80), ((3, 3, 15, 2, 6), 9, 90)], 3, 300, False),
         _prot([((1, 10, 5, 1, 1), 10, 100), ((3, 2, 10, 1, 4), 11, 110), ((3, 3, 15, 1, 4), 12, 120)], 4, 400,
               True)],
    ],
    expect={
        (0, 0): dict(Ke=_KE_AB, Kmf=0.5, Kmb=0.5 * _KE_AB, Vmax=2.0, N=_vec((0, -1), (1, 1)), Nf=_vec((0, 1)),
                     Nb=_vec((1, 1)), A=_vec((2, 1), (3, -2)), Kmr={2: 1.0, 3: 2.0**-2}),
        (0, 1): dict(Ke=_KE_AB, Kmf=0.5, Kmb=0.5 * _KE_AB, Vmax=2.0, N=_vec((0, -1), (1, 1)), Nf=_vec((0, 1)),
                     Nb=_vec((1, 1)), A=_vec((0, 1), (4, 3)), Kmr={0: 1.0, 4: 1.5**3}),
        (0, 2): dict(Kmf=0.0, Kmb=0.0, Vmax=0.0, N=_vec(), Nf=_vec(), Nb=_vec(), A=_vec()),
        (1, 0): dict(Ke=_KE_AB, Kmf=0.5, Kmb=0.5 * _KE_AB, Vmax=2.0, N=_vec((0, -1), (1, 1)), Nf=_vec((0, 1)),
                     Nb=_vec((1, 1)), A=_vec((1, -1), (5, -3)), Kmr={1: 1.0, 5: 1.5**-3}),
        (1, 1): dict(Ke=_KE_AB, Kmf=0.5, Kmb=0.5 * _KE_AB, Vmax=2.0, N=_vec((0, -1), (1, 1)), Nf=_vec((0, 1)),
                     Nb=_vec((1, 1)), A=_vec((3, 5)), Kmr={3: _mean(1.0, 1.5) ** 5}),
        (1, 2): dict(Kmf=0.0, Kmb=0.0, Vmax=0.0, N=_vec(), Nf=_vec(), Nb=_vec(), A=_vec()),
    },
)

_KE00, _KE01, _KE02 = _ke([_a, _d], [_b, _b, _c]), _ke([_b, _d], [_c, _b, _c]), _ke([_d], [_b, _b])
_KE10, _KE11 = _ke([_b, _d], [_a, _b, _c]), _ke([_b, _b, _c], [_c, _d])
CATALYTIC = dict(
    cells=[
        [_prot([((1, 1, 5, 1, 1), 1, 10), ((1, 2, 15, 2, 3), 2, 20)], 1, 100, False),
         _prot([((1, 10, 9, 1, 2), 3, 30), ((1, 3, 12, 2, 3), 4, 40)], 2, 200, True),
         _prot([((1, 19, 29, 1, 4), 5, 50)], 3, 300, False)],
        [_prot([((1, 1, 3, 2, 1), 6, 60), ((1, 11, 14, 2, 3), 7, 70)], 4, 400, True),
         _prot([((1, 9, 3, 1, 2), 8, 80), ((1, 13, 17, 1, 3), 9, 90)], 5, 500, False)],
    ],
    expect={
        (0, 0): dict(Ke=_KE00, Kmf=_mean(0.5, 1.5) / _KE00, Kmb=_mean(0.5, 1.5), Vmax=_mean(1.1, 1.2),
                     N=_vec((0, -1), (1, 2), (2, 1), (3, -1)), Nf=_vec((0, 1), (3, 1)), Nb=_vec((1, 2), (2, 1))),
        (0, 1): dict(Ke=_KE01, Kmf=_mean(0.9, 1.2) / _KE01, Kmb=_mean(0.9, 1.2), Vmax=_mean(2.0, 1.3),
                     N=_vec((2, 2), (3, -1)), Nf=_vec((1, 1), (3, 1)), Nb=_vec((1, 1), (2, 2))),
        (0, 2): dict(Ke=_KE02, Kmf=2.9 / _KE02, Kmb=2.9, Vmax=2.9, N=_vec((1, 2), (3, -1)), Nf=_vec((3, 1)),
                     Nb=_vec((1, 2))),
        (1, 0): dict(Ke=_KE10, Kmf=_mean(0.3, 1.4) / _KE10, Kmb=_mean(0.3, 1.4), Vmax=_mean(1.1, 2.1),
                     N=_vec((0, 1), (2, 1), (3, -1)), Nf=_vec((1, 1), (3, 1)), Nb=_vec((0, 1), (1, 1), (2, 1))),
        (1, 1): dict(Ke=_KE11, Kmf=_mean(0.3, 1.7), Kmb=_mean(0.3, 1.7) * _KE11, Vmax=_mean(1.9, 2.3),
                     N=_vec((1, -2), (3, 1)), Nf=_vec((1, 2), (2, 1)), Nb=_vec((2, 1), (3, 1))),
        (1, 2): dict(Kmf=0.0, Kmb=0.0, Vmax=0.0, N=_vec(), Nf=_vec(), Nb=_vec()),
    },
    A_zero=True,
)

CASES = {"transporter": TRANSPORTER, "regulatory": REGULATORY, "catalytic": CATALYTIC}


def _build(case, device):
    kin = _kinetics(device)
    # the reference assigns zero tensors and reads them back after set_cell_params
    params = {n: torch.zeros(2, 3, 8, dtype=torch.int32, device=device) for n in ("N", "Nf", "Nb", "A")}
    params["Kmr"] = torch.zeros(2, 3, 8, dtype=torch.float32, device=device)
    params.update({n: torch.zeros(2, 3, dtype=torch.float32, device=device) for n in ("Ke", "Kmf", "Kmb", "Vmax")})
    for n, t in params.items():
        setattr(kin, n, t)
    kin.set_cell_params(cell_idxs=[0, 1], proteomes=case["cells"])
    return kin, {n: getattr(kin, n).cpu() for n in params}


def _check(case, got):
    for (c, p), exp in case["expect"].items():
        for name in ("Ke", "Kmf", "Kmb", "Vmax"):
            if name in exp:
                assert got[name][c, p].item() == pytest.approx(exp[name], abs=_TOL, rel=_TOL), (c, p, name)
        for name in ("N", "Nf", "Nb", "A"):
            if name in exp:
                assert got[name][c, p].tolist() == exp[name], (c, p, name)
        for j, v in exp.get("Kmr", {}).items():
            assert got["Kmr"][c, p, j].item() == pytest.approx(v, abs=_TOL, rel=_TOL), (c, p, "Kmr", j)
    if case.get("A_zero"):
        assert (got["A"] == 0).all()
        assert (got["Kmr"] - 1.0 < _TOL).all()


@pytest.mark.parametrize("name", list(CASES))
def test_cell_params_match_reference_fixture(name):
    case = CASES[name]
    kin, got = _build(case, "cpu")
    _check(case, got)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_cell_params_match_reference_fixture_on_gpu(name):
    case = CASES[name]
    kin, got = _build(case, "cuda")
    _check(case, got)


def test_proteome_views_of_reference_fixtures():
    """Kinetics.get_proteome on the fixture proteomes (the reference asserts every domain view)."""
    kin = _kinetics()
    views = kin.get_proteome(TRANSPORTER["cells"][1])
    p0, p1 = views
    assert (p0.cds_start, p0.cds_end, p0.is_fwd) == (91, 112, False)
    assert [type(d).__name__ for d in p0.domains] == ["TransporterDomain"] * 4
    assert [d.molecule for d in p0.domains] == [_a, _a, _b, _c]
    assert [round(d.vmax, 4) for d in p0.domains] == [1.5, 1.4, 1.3, 1.2]
    assert [round(d.km, 4) for d in p0.domains] == [0.4, 0.5, 0.6, 0.7]
    assert [(d.start, d.end) for d in p0.domains] == [(1, 10), (2, 20), (3, 30), (4, 40)]
    assert isinstance(p1.domains[0], ms.CatalyticDomain)
    assert p1.domains[0].substrates == [_a] and p1.domains[0].products == [_b]
    assert p1.domains[0].vmax == pytest.approx(2.0, abs=_TOL) and p1.domains[0].km == pytest.approx(0.5, abs=_TOL)
    c0, c1 = kin.get_proteome(REGULATORY["cells"][0]), kin.get_proteome(REGULATORY["cells"][1])
    regs = [c0[0].domains[1], c0[0].domains[2], c0[1].domains[1], c0[1].domains[2], c1[0].domains[1],
            c1[0].domains[2], c1[1].domains[1], c1[1].domains[2]]
    assert [d.effector for d in regs] == [_c, _d, _a, _a, _b, _b, _d, _d]
    assert [d.is_inhibiting for d in regs] == [False, True, False, False, True, True, False, False]
    assert [d.is_transmembrane for d in regs] == [False, False, False, True, False, True, False, False]
    assert [d.hill for d in regs] == [1, 2, 1, 3, 1, 3, 2, 3]
    assert [round(d.km, 4) for d in regs] == [1.0, 2.0, 1.0, 1.5, 1.0, 1.5, 1.0, 1.5]
    cat = kin.get_proteome(CATALYTIC["cells"][0])
    assert cat[0].domains[1].substrates == [_d] and cat[0].domains[1].products == [_b, _c]  # bwd bc->d
    assert cat[2].domains[0].substrates == [_d] and cat[2].domains[0].products == [_b, _b]


# ------------------------------------------------------------------------------------ helpers
def test_multiply_signals_reference_cases():
    """reference tests/fast/test_kinetics.py:1697-1775: products of x^n over involved signals,
    Inf -> _MAX, an involved zero -> 0, the involvement mask."""
    kin = _kinetics()
    X = torch.tensor([[1.0, 2.0, 3.0, 4.0], [100.0, 200.0, 300.0, 400.0], [0.0, 0.0, 3.0, 4.0], [0.0, 0.0, 0.0, 0.0]])
    N = torch.tensor([
        [[0, 1, 2, 0], [3, 0, 0, 0], [0, 0, 0, 0]],
        [[10, 10, 5, 0], [0, 0, 0, 0], [0, 0, 0, 0]],
        [[2, 1, 2, 0], [0, 0, 1, 2], [0, 0, 0, 0]],
        [[1, 1, 1, 1], [1, 2, 0, 0], [0, 0, 0, 0]],
    ], dtype=torch.int32)
    xx, prots = kin._multiply_signals(X=X, N=N)
    assert xx.size() == (4, 3) and prots.size() == (4, 3)
    assert prots.tolist() == [[True, True, False], [True, False, False], [True, True, False], [True, True, False]]
    assert xx[0, 0] == X[0, 1] * X[0, 2] ** 2
    assert xx[0, 1] == X[0, 0] ** 3
    assert xx[1, 0] == MAX
    assert xx[2, 0] == 0.0
    assert xx[2, 1] == X[2, 3] ** 2 * X[2, 2]
    assert xx[3, 0] == 0.0 and xx[3, 1] == 0.0


def test_get_quotient_reference_cases():
    """reference tests/fast/test_kinetics.py:1778-1853: Q = prod(products) / prod(substrates) with
    _MAX / _MAX = 1, a missing substrate -> _MAX, a missing product -> _EPS, 0 / 0 -> 1."""
    kin = _kinetics()
    X = torch.tensor([[1.0, 2.0, 3.0, 4.0], [100.0, 200.0, 300.0, 400.0], [0.0, 0.0, 10.0, 20.0]])
    kin.Nf = torch.tensor([
        [[1, 0, 0, 0], [0, 1, 0, 1], [0, 2, 1, 0]],
        [[5, 7, 0, 0], [0, 0, 20, 0], [1, 0, 0, 0]],
        [[1, 0, 3, 0], [0, 0, 1, 0], [1, 0, 0, 0]],
    ], dtype=torch.int32)
    kin.Nb = torch.tensor([
        [[0, 1, 0, 0], [0, 0, 1, 0], [3, 0, 0, 0]],
        [[0, 0, 10, 0], [0, 0, 0, 30], [0, 0, 0, 0]],
        [[0, 0, 0, 2], [2, 0, 0, 0], [0, 1, 0, 0]],
    ], dtype=torch.int32)
    Q = kin._get_quotient(X=X)
    x = X[0]
    assert Q[0, 0] == x[1] / x[0]
    assert Q[0, 1] == x[2] / (x[1] * x[3])
    assert Q[0, 2] == x[0] ** 3 / (x[1] ** 2 * x[2])
    x = X[1]
    assert Q[1, 0] == x[2] ** 10 / (x[0] ** 5 * x[1] ** 7)
    assert Q[1, 1] == 1.0
    assert Q[2, 0] == MAX
    assert Q[2, 1] == EPS
    assert Q[2, 2] == 1.0
