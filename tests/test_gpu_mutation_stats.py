"""Statistics of the HIP mutation kernels against the reference's generative model (GPU).

Reference semantics (``rust/mutations.rs``): point mutations draw ``Poisson(p * len)`` distinct
positions per genome (``:11-29``); each is an indel with probability ``p_indel`` -- a deletion with
``p_del``, else an insertion of a random nucleotide -- and otherwise a substitution by a random
nucleotide, which may repeat the old one (``:30-60``). Recombination draws ``Poisson(p * (n0 + n1))``
strand breaks per pair, shuffles the pieces and splits them into two genomes, conserving the total
(``:78-154``). The kernels (``csrc/hip/mutations.hip`` ``mut_count`` / ``mut_apply`` / ``rec_count``
/ ``rec_apply``) run here on 50k synthetic genomes; every rate and share is checked at 5 sigma.
"""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, L = 50_000, 1_000


def _m():
    from magicsoup_amd.ops import native

    return native.hip()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _genomes(n: int, length: int, seed: int) -> torch.Tensor:
    g = torch.Generator(device="cuda").manual_seed(seed)
    lut = torch.tensor(list(b"TCGA"), dtype=torch.uint8, device="cuda")
    return lut[torch.randint(0, 4, (n, length), device="cuda", generator=g)].contiguous()


def _within(got: float, want: float, sd: float, what: str) -> None:
    assert abs(got - want) <= 5 * sd, f"{what}: {got:.5f} vs {want:.5f} (5 sd = {5 * sd:.5f})"


def _binom(hits: int, n: int, p: float, what: str) -> None:
    _within(hits / n, p, math.sqrt(p * (1 - p) / n), what)


def _offsets(n: int, length: int) -> torch.Tensor:
    """Per-genome byte offsets of rows laid out back to back (the kernels read genome i at
    pool + off[i], models/strings.py PoolArena)."""
    return (torch.arange(n, dtype=torch.int64, device="cuda") * length).contiguous()


def _point_mutations(p: float, p_indel: float, p_del: float, seed: int):
    data = _genomes(N, L, seed)
    off = _offsets(N, L)
    lens = torch.full((N,), L, dtype=torch.int32, device="cuda")
    k = torch.empty(N, dtype=torch.int32, device="cuda")
    m = _m()
    m.mut_count(N, 0, lens.data_ptr(), p, seed, 7, k.data_ptr(), 0, 0, 0, _stream())
    sel = torch.nonzero(k > 0).flatten().contiguous()
    nsel = int(sel.numel())
    out_w = L + int(k.max().item()) + 16
    out = torch.zeros(nsel, out_w, dtype=torch.uint8, device="cuda")
    out_len = torch.empty(nsel, dtype=torch.int32, device="cuda")
    m.mut_apply(nsel, 0, sel.data_ptr(), 0, data.data_ptr(), off.data_ptr(), lens.data_ptr(), k.data_ptr(), p_indel,
                p_del, seed, 7,
                out.data_ptr(), out_w, out_len.data_ptr(), _stream())
    torch.cuda.synchronize()
    return data.cpu().numpy(), k.cpu().numpy(), sel.cpu().numpy(), out.cpu().numpy(), out_len.cpu().numpy()


def test_point_mutation_counts_are_poisson():
    p = 1e-3  # lambda = 1 per genome
    _, k, _, _, _ = _point_mutations(p, 0.4, 0.66, seed=11)
    lam = p * L
    _within(float(k.mean()), lam, math.sqrt(lam / N), "mean events per genome")
    # Poisson: variance = mean; var of the sample variance ~ (mu4 - sigma^4) / n = (lam + 2 lam^2) / n
    _within(float(k.var()), lam, math.sqrt((lam + 2 * lam * lam) / N), "variance of events per genome")
    _binom(int((k == 0).sum()), N, math.exp(-lam), "P(no event)")


def test_point_mutation_event_kinds_and_shares():
    p_indel, p_del = 0.4, 0.66
    data, k, sel, out, out_len = _point_mutations(1e-3, p_indel, p_del, seed=12)
    one = np.nonzero(k[sel] == 1)[0]  # genomes with exactly one event: its kind is readable
    delta = out_len[one] - L
    n1 = len(one)
    assert n1 > 15_000
    _binom(int((delta == -1).sum()), n1, p_indel * p_del, "deletion share")
    _binom(int((delta == 1).sum()), n1, p_indel * (1 - p_del), "insertion share")
    assert set(np.unique(delta).tolist()) <= {-1, 0, 1}
    subs_pos, same = [], 0
    n_sub = 0
    for j in one:
        orig, new = data[sel[j]], out[j, : out_len[j]]
        d = int(out_len[j]) - L
        if d == 0:
            diff = np.nonzero(orig != new)[0]
            assert len(diff) <= 1
            n_sub += 1
            if len(diff) == 0:
                same += 1  # the substitute repeated the old nucleotide (reference quirk, kept)
            else:
                subs_pos.append(int(diff[0]))
        elif d == -1:  # one base removed, everything else in order
            i = int(np.argmax(orig[:-1] != new)) if (orig[:-1] != new).any() else L - 1
            assert np.array_equal(orig[:i], new[:i]) and np.array_equal(orig[i + 1 :], new[i:])
        else:  # one base inserted
            i = int(np.argmax(orig != new[:-1])) if (orig != new[:-1]).any() else L
            assert np.array_equal(orig[:i], new[:i]) and np.array_equal(orig[i:], new[i + 1 :])
    _binom(same, n_sub, 0.25, "substitutions that keep the nucleotide")
    # substitution positions are uniform over the genome (10 bins, chi-square at ~5 sd)
    hist = np.bincount(np.array(subs_pos) * 10 // L, minlength=10)
    exp = len(subs_pos) / 10
    chi2 = float(((hist - exp) ** 2 / exp).sum())
    assert chi2 < 9 + 5 * math.sqrt(18), f"positions not uniform: chi2 = {chi2:.1f}"


def test_point_mutation_length_change_matches_model():
    """All genomes, any number of events: E[length change] = events * p_indel * (1 - 2 p_del)."""
    p_indel, p_del = 0.4, 0.66
    _, k, sel, _, out_len = _point_mutations(2e-3, p_indel, p_del, seed=13)
    events = int(k.sum())
    per = p_indel * (1 - 2 * p_del)
    var = p_indel - per * per  # E[d^2] - E[d]^2 per event (d in {-1, 0, +1})
    delta = float((out_len - L).sum())
    _within(delta / events, per, math.sqrt(var / events), "mean length change per event")


@pytest.mark.parametrize("p_del", [0.0, 1.0])
def test_pure_insertions_and_deletions(p_del):
    _, k, sel, _, out_len = _point_mutations(1e-3, 1.0, p_del, seed=14)
    want = L + (-1 if p_del == 1.0 else 1) * k[sel]
    assert np.array_equal(out_len, want)


def test_recombination_breaks_and_conservation():
    p = 5e-4  # lambda = p * 2L = 1 break per pair
    n_pairs = N // 2
    data = _genomes(2 * n_pairs, L, seed=21)
    off = _offsets(2 * n_pairs, L)
    lens = torch.full((2 * n_pairs,), L, dtype=torch.int32, device="cuda")
    pairs = torch.arange(2 * n_pairs, dtype=torch.int32, device="cuda").view(n_pairs, 2).contiguous()
    k = torch.empty(n_pairs, dtype=torch.int32, device="cuda")
    m = _m()
    m.rec_count(n_pairs, pairs.data_ptr(), lens.data_ptr(), p, 21, 3, k.data_ptr(), _stream())
    kk = k.cpu().numpy()
    lam = p * 2 * L
    _within(float(kk.mean()), lam, math.sqrt(lam / n_pairs), "mean strand breaks per pair")
    _within(float(kk.var()), lam, math.sqrt((lam + 2 * lam * lam) / n_pairs), "variance of strand breaks")
    sel = torch.nonzero(k > 0).flatten().contiguous()
    nsel = int(sel.numel())
    out_w = 2 * L
    parts_cap = int(k.max().item()) + 2
    out = torch.zeros(2 * nsel, out_w, dtype=torch.uint8, device="cuda")
    out_len = torch.empty(2 * nsel, dtype=torch.int32, device="cuda")
    out_rows = torch.empty(2 * nsel, dtype=torch.int64, device="cuda")
    parts = torch.empty(nsel * parts_cap * 3, dtype=torch.int32, device="cuda")
    m.rec_apply(nsel, 0, sel.data_ptr(), pairs.data_ptr(), 0, data.data_ptr(), off.data_ptr(), lens.data_ptr(),
                k.data_ptr(), 21, 3,
                parts.data_ptr(), parts_cap, out.data_ptr(), out_w, out_len.data_ptr(), out_rows.data_ptr(), _stream())
    torch.cuda.synchronize()
    d, o, ol, rows, s = data.cpu().numpy(), out.cpu().numpy(), out_len.cpu().numpy(), out_rows.cpu().numpy(), sel.cpu().numpy()
    changed = 0
    for j in range(nsel):
        a, b = 2 * int(s[j]), 2 * int(s[j]) + 1
        assert rows[2 * j] == a and rows[2 * j + 1] == b
        na, nb = int(ol[2 * j]), int(ol[2 * j + 1])
        assert na + nb == 2 * L  # total length conserved
        ga, gb = o[2 * j, :na], o[2 * j + 1, :nb]
        # the pieces are rearranged, never altered: base composition of the pair is conserved
        cin = np.bincount(np.concatenate([d[a], d[b]]), minlength=256)
        cout = np.bincount(np.concatenate([ga, gb]), minlength=256)
        assert np.array_equal(cin, cout)
        changed += not (na == L and np.array_equal(ga, d[a]) and np.array_equal(gb, d[b]))
    assert changed > 0.5 * nsel
