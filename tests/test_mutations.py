"""Point mutations and recombinations (reference tests/fast/test_mutations.py behaviours), for the
list API (host core) and the in-arena world path."""
import torch

import magicsoup_amd as ms
from magicsoup_amd.models import mutations as muts


def test_substitutions_keep_length_and_rate():
    seqs = ["GGGGGGGGGGGGGGGGGGGG"] * 300
    out = muts.point_mutations(seqs=seqs, p=0.05, p_indel=0.0)
    # P(at least one event in 20 bp at 5%) = 64%
    assert 120 < len(out) < 260
    assert all(len(s) == 20 for s, _ in out)
    assert all(0 <= i < 300 for _, i in out)
    assert len({i for _, i in out}) == len(out)
    # a substitution draws uniformly from all 4 nucleotides, so 3/4 change the base
    changed = sum(s != "G" * 20 for s, _ in out)
    assert changed > 0.6 * len(out)


def test_deletions_shorten_and_insertions_lengthen():
    seqs = ["ACGTACGTAC"] * 200
    dels = muts.point_mutations(seqs=seqs, p=0.1, p_indel=1.0, p_del=1.0)
    assert len(dels) > 100 and all(len(s) < 10 for s, _ in dels)
    ins = muts.point_mutations(seqs=seqs, p=0.1, p_indel=1.0, p_del=0.0)
    assert len(ins) > 100 and all(len(s) > 10 for s, _ in ins)
    assert all(set(s) <= set("ACGT") for s, _ in ins)


def test_no_mutations_at_zero_rate_and_empty_inputs():
    assert muts.point_mutations(seqs=["ACGT"] * 50, p=0.0) == []
    assert muts.point_mutations(seqs=[], p=0.5) == []
    assert muts.point_mutations(seqs=[""] * 10, p=0.5) == []
    assert muts.recombinations(seq_pairs=[], p=0.5) == []


def test_indices_refer_to_input_positions():
    seqs = ["A" * 50, "", "C" * 50, "", "G" * 50]
    out = muts.point_mutations(seqs=seqs, p=0.5, p_indel=0.0)
    assert {i for _, i in out} <= {0, 2, 4}


def test_recombinations_conserve_material():
    pair = ("TTTTTTTTTTTT", "GGGGGGGGGGGG")
    out = muts.recombinations(seq_pairs=[pair] * 200, p=0.1)
    assert len(out) > 120
    for a, b, i in out:
        assert len(a) + len(b) == 24
        assert sorted(a + b) == sorted(pair[0] + pair[1])
        assert 0 <= i < 200
    mixed = sum(("G" in a) or ("T" in b) for a, b, _ in out)
    assert mixed > 0.5 * len(out)


def test_recombinations_with_empty_partners():
    pairs = [("CCCCAAAA", ""), ("", "CCCCAAAA"), ("CC", "AA")]
    out = muts.recombinations(seq_pairs=pairs, p=1.0)
    assert len(out) == 3
    for a, b, i in out:
        assert sorted(a + b) == sorted(pairs[i][0] + pairs[i][1])


def test_world_mutations_change_arena_and_params():
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    ms.set_seed(4)
    w = ms.World(chemistry=CHEMISTRY, map_size=16, seed=4)
    w.spawn_cells([ms.random_genome(300) for _ in range(100)])
    before = list(w.cell_genomes)
    w.mutate_cells(p=0.02)
    after = list(w.cell_genomes)
    assert sum(a != b for a, b in zip(before, after)) > 80
    # params equal a fresh translation of the mutated genomes
    N = w.kinetics.N.clone()
    w.update_cells([(g, i) for i, g in enumerate(after)])
    p = min(N.size(1), w.kinetics.N.size(1))
    assert torch.equal(N[:, :p], w.kinetics.N[:, :p])
    # only selected cells mutate
    w.mutate_cells(cell_idxs=[0, 1, 2], p=0.5)
    now = list(w.cell_genomes)
    assert now[3:] == after[3:]


def test_world_recombination_pairs_neighbours_only():
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    w = ms.World(chemistry=CHEMISTRY, map_size=12, seed=9)
    w.spawn_cells([ms.random_genome(200) for _ in range(4)])
    w.cell_map = torch.zeros(12, 12, dtype=torch.bool)
    w.cell_positions = torch.tensor([[0, 0], [0, 1], [6, 6], [6, 8]], dtype=torch.int32)
    w.cell_map[w.cell_positions[:, 0].long(), w.cell_positions[:, 1].long()] = True
    g = list(w.cell_genomes)
    w.recombinate_cells(p=0.5)
    h = list(w.cell_genomes)
    # cells 2 and 3 are 2 pixels apart: untouched; 0 and 1 are neighbours: material exchanged
    assert h[2:] == g[2:]
    assert len(h[0]) + len(h[1]) == 400
    assert (h[0], h[1]) != (g[0], g[1])


def test_list_api_inputs_read_in_place_are_left_untouched():
    # the host core reads str inputs in place: outputs are fresh strings, the inputs never change,
    # and pairs may be given as lists as well as tuples
    seqs = ["ACGT" * 50 for _ in range(200)]
    before = list(seqs)
    out = muts.point_mutations(seqs=seqs, p=0.05)
    assert out and seqs == before
    pairs = [["A" * 40, "C" * 40] for _ in range(100)]
    rec = muts.recombinations(seq_pairs=pairs, p=0.1)
    assert rec and all(p == ["A" * 40, "C" * 40] for p in pairs)
    for s0, s1, i in rec:
        assert sorted(s0 + s1) == sorted("A" * 40 + "C" * 40) and 0 <= i < 100


def test_get_neighbors_returns_int_tuples():
    w = ms.World(chemistry=ms.Chemistry(molecules=[ms.Molecule("nbtest_a", 10.0)], reactions=[]), map_size=8)
    w.spawn_cells(genomes=["ACGT" * 20] * 30)
    pairs = w.get_neighbors(cell_idxs=list(range(w.n_cells)))
    assert pairs and all(type(p) is tuple and len(p) == 2 and type(p[0]) is int and p[0] < p[1] for p in pairs)
    assert len(set(pairs)) == len(pairs)
