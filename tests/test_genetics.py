"""Genetics: CDS scan, domain extraction, translation (reference tests/fast/test_genetics.py).

The native scan (csrc/include/ms_common.h, shared by the host core and the HIP kernel) is checked
against a direct Python transcription of the reference's algorithm (rust/genetics.rs:13-123:
per-frame stacks of open start codons popped at the next in-frame stop) on random sequences, plus
hand-checked fixtures."""
import random

import pytest

import magicsoup_amd as ms
from magicsoup_amd.constants import CODON_SIZE
from magicsoup_amd.ops import native

STARTS = ["TTG", "GTG", "ATG"]
STOPS = ["TGA", "TAG", "TAA"]
_COMP = {"A": "T", "T": "A", "C": "G", "G": "C"}


def _revcomp(seq: str) -> str:
    return "".join(_COMP[c] for c in reversed(seq))


def _oracle_cdss(seq: str, min_size: int, starts=STARTS, stops=STOPS) -> list[tuple[int, int]]:
    """Reference order: in order of stop codons; per stop, the latest start first."""
    out = []
    open_starts: list[list[int]] = [[], [], []]
    for i in range(len(seq) - CODON_SIZE + 1):
        codon = seq[i : i + CODON_SIZE]
        f = i % CODON_SIZE
        if codon in starts:
            open_starts[f].append(i)
        elif codon in stops:
            while open_starts[f]:
                s = open_starts[f].pop()
                if i + CODON_SIZE - s >= min_size:
                    out.append((s, i + CODON_SIZE))
    return out


def _oracle_domains(seq, start, end, dom_size, dts, dom_types, one, two):
    doms, i, useful = [], 0, False
    while i + dom_size <= end - start:
        s0 = start + i
        t = dom_types.get(seq[s0 : s0 + dts], 0)
        if t:
            a = s0 + dts
            spec = (t, one.get(seq[a : a + 3], 0), one.get(seq[a + 3 : a + 6], 0), one.get(seq[a + 6 : a + 9], 0),
                    two.get(seq[a + 9 : a + 15], 0))
            doms.append((spec, i, i + dom_size))
            useful |= t != 3
            i += dom_size
        else:
            i += CODON_SIZE
    return doms, useful


def _oracle_translate(genome: str, g: ms.Genetics):
    prots = []
    for seq, fwd in ((genome, True), (_revcomp(genome), False)):
        for s, e in _oracle_cdss(seq, g.dom_size, g.start_codons, g.stop_codons):
            doms, useful = _oracle_domains(seq, s, e, g.dom_size, g.dom_type_size, g.domain_map, g.one_codon_map,
                                           g.two_codon_map)
            if useful:
                prots.append((doms, s, e, fwd))
    return prots


def _norm(prots):
    return [([(tuple(d[0]), d[1], d[2]) for d in doms], s, e, bool(f)) for doms, s, e, f in prots]


# --------------------------------------------------------------------------------------------- tests
@pytest.mark.parametrize("seq", ["ACTGG", "", "A", "TTTTCCCCGGGGAAAA", "random101"])
def test_reverse_complement(seq):
    if seq == "random101":  # drawn at run time so parametrize ids stay stable under pytest-xdist
        seq = ms.random_genome(101)
    assert native.host().reverse_complement(seq) == _revcomp(seq)


@pytest.mark.parametrize(
    "seq, exp",
    [
        # start at 0, stop TGA at 15: exactly the minimum size of 18
        ("TTGAAAGAGCAAATTTGA", [(0, 18)]),
        # too short by one codon
        ("TTGAAAGAGCAATGA", []),
        # two starts in one frame close at the same stop, latest start first
        ("ATGCCCGTGCCCAAACCCGGGTAA", [(6, 24), (0, 24)]),
        # starts in different frames reach different stops
        ("GTGTGCTCGAAAGAGAACGCAAATTCGTAACCTAG", [(0, 30), (2, 35)]),
        # a stop before the start closes nothing
        ("TAAATGCCCCCCCCCCCCCCCTAG", [(3, 24)]),
    ],
)
def test_coding_regions_fixtures(seq, exp):
    res = native.host().get_coding_regions(seq, 18, STARTS, STOPS, True)
    assert [(s, e) for s, e, _ in res] == exp
    assert all(f is True for *_, f in res)
    assert _oracle_cdss(seq, 18) == exp


@pytest.mark.parametrize("seed", range(6))
def test_coding_regions_match_reference_algorithm(seed):
    rng = random.Random(seed)
    for _ in range(40):
        seq = "".join(rng.choice("TCGA") for _ in range(rng.randint(0, 400)))
        min_size = rng.choice([6, 18, 48])
        res = native.host().get_coding_regions(seq, min_size, STARTS, STOPS, False)
        assert [(s, e) for s, e, _ in res] == _oracle_cdss(seq, min_size)
        assert all(f is False for *_, f in res)


def test_extract_domains_hand_checked():
    dom_types = {"AAA": 1, "GGG": 2, "CCC": 3}
    one = {"ACT": 1, "CTG": 2, "CCG": 3, "GGA": 4, "TGT": 5}
    two = {"ACTGAT": 1, "CTGTAT": 2, "CCGCGA": 3, "GGAATC": 4, "TGTCGA": 5}
    dts = 3
    ds = dts + 5 * CODON_SIZE  # 18
    # catalytic domain 3 codons into the CDS, then filler
    cds0 = "TTT" + "AAA" + "CTG" + "TGT" + "ACT" + "CCGCGA" + "TTTTTT"
    # only a regulatory domain -> protein dropped
    cds1 = "CCC" + "GGA" + "GGA" + "GGA" + "TGTCGA" + "TTT"
    # two back-to-back domains; the GGG right after the first type codon is its first token (unmapped: 0)
    cds2 = "GGG" + "GGG" + "ACT" + "ACT" + "CTGTAT" + "CCC" + "ACT" + "CTG" + "CCG" + "GGAATC"
    genome = cds0 + cds1 + cds2
    b0, b1 = len(cds0), len(cds0) + len(cds1)
    cdss = [(0, b0, True), (b0, b1, False), (b1, len(genome), True)]
    res = native.host().extract_domains(genome, cdss, ds, dts, dom_types, one, two)
    got = _norm(res)
    assert got == [
        ([((1, 2, 5, 1, 3), 3, 3 + ds)], 0, b0, True),
        ([((2, 0, 1, 1, 2), 0, ds), ((3, 1, 2, 3, 4), ds, 2 * ds)], b1, len(genome), True),
    ]
    for (doms, s, e, _), (odoms, *_rest) in zip(got, [_oracle_domains(genome, s, e, ds, dts, dom_types, one, two) + (0,)
                                                         for s, e, _ in (cdss[0], cdss[2])]):
        assert doms == [(tuple(d[0]), d[1], d[2]) for d in odoms]


@pytest.mark.parametrize("seed", range(3))
def test_translation_matches_reference_algorithm(seed):
    random.seed(seed)
    g = ms.Genetics()
    rng = random.Random(100 + seed)
    genomes = ["".join(rng.choice("TCGA") for _ in range(rng.randint(0, 1200))) for _ in range(60)]
    res = g.translate_genomes(genomes)
    assert len(res) == len(genomes)
    for genome, prots in zip(genomes, res):
        assert _norm(prots) == _norm(_oracle_translate(genome, g))


def test_translation_tokens_agree_with_lists():
    """The dense token path (what the parameter builder consumes) carries the same proteomes."""
    from magicsoup_amd.models.strings import pack_strings

    g = ms.Genetics()
    genomes = [ms.random_genome(s) for s in (0, 30, 300, 900, 900, 2000)]
    lists = g.translate_genomes(genomes)
    arr, lens = pack_strings(genomes)
    tokens, nprot = g.tables.translate_tokens(arr, lens)
    import numpy as np

    tokens, nprot = np.asarray(tokens), np.asarray(nprot)
    for k, prots in enumerate(lists):
        assert nprot[k] == len(prots)
        for p, (doms, *_rest) in enumerate(prots):
            for d, (spec, *_r) in enumerate(doms):
                assert tuple(tokens[k, p, d]) == tuple(spec)
            assert not tokens[k, p, len(doms) :].any()


def test_genetics_maps_are_consistent():
    g = ms.Genetics()
    # token codons never contain a stop codon (a premature stop would end the CDS)
    assert set(g.one_codon_map) == {c for c in ms.codons(n=1) if c not in g.stop_codons}
    assert sorted(g.one_codon_map.values()) == list(range(1, len(g.one_codon_map) + 1))
    assert all(k[:3] not in g.stop_codons for k in g.two_codon_map)
    # domain-type prefixes avoid start codons (reference genetics.py:95)
    assert all(len(k) == g.dom_type_size for k in g.domain_map)
    assert set(g.domain_map.values()) <= {1, 2, 3}
    assert all(not any(k[i : i + 3] in g.start_codons for i in range(0, len(k), 3)) for k in g.domain_map)
    assert g.dom_size == g.dom_type_size + 5 * CODON_SIZE


def test_genetics_rejects_too_small_type_space():
    with pytest.warns(UserWarning):
        ms.Genetics(n_dom_type_codons=1)


def _count_types(proteomes):
    cnt = {1: 0, 2: 0, 3: 0}
    for cell in proteomes:
        for doms, *_ in cell:
            for spec, *_r in doms:
                cnt[spec[0]] += 1
    return cnt


@pytest.mark.slow
def test_domain_type_frequencies_follow_probabilities():
    genomes = [ms.random_genome(s=500) for _ in range(800)]
    c = _count_types(ms.Genetics(p_catal_dom=0.1, p_transp_dom=0.1, p_reg_dom=0.1).translate_genomes(genomes))
    n = sum(c.values())
    assert abs(c[1] - c[2]) < 0.1 * n
    c = _count_types(ms.Genetics(p_catal_dom=0.01, p_transp_dom=0.1, p_reg_dom=0.1).translate_genomes(genomes))
    n = sum(c.values())
    assert c[2] - c[1] > 0.25 * n
