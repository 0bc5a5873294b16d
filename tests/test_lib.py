"""The reference's direct native surface (``from magicsoup import _lib``, rust/lib.rs:182-202),
exercised the way the reference's tests call it (tests/fast/test_genetics.py:62-93)."""
import magicsoup as ms
from magicsoup import _lib
from magicsoup.constants import CODON_SIZE


def test_lib_exposes_the_reference_functions():
    names = {"dist_1d", "free_moores_nghbhd", "point_mutations", "recombinations", "get_coding_regions",
             "extract_domains", "reverse_complement", "translate_genomes", "get_neighbors",
             "divide_cells_if_possible", "move_cells", "get_proteome"}
    assert names <= set(dir(_lib))


def test_lib_genetics_reference_cases():
    assert _lib.reverse_complement("ACTGG") == "CCAGT"
    # reference tests/fast/test_genetics.py:_DATA[2] and [3] (reverse-strand flag as in the test)
    res = _lib.get_coding_regions("TTGAAAGAGCAAATTTGA", 18, ["TTG", "GTG", "ATG"], ["TGA", "TAG", "TAA"], False)
    assert [(a, b) for a, b, _ in res] == [(0, 18)] and not res[0][2]
    res = _lib.get_coding_regions("GTGTGCTCGAAAGAGAACGCAAATTCGTAACCTAG", 18, ["TTG", "GTG", "ATG"],
                                  ["TGA", "TAG", "TAA"], True)
    assert {(a, b) for a, b, _ in res} == {(0, 30), (2, 35)}
    # reference tests/fast/test_genetics.py:test_extract_domains (cds 0 and 4)
    dom_type_map = {"AAA": 1, "GGG": 2, "CCC": 3}
    two = {"ACTGAT": 1, "CTGTAT": 2, "CCGCGA": 3, "GGAATC": 4, "TGTCGA": 5}
    one = {"ACT": 1, "CTG": 2, "CCG": 3, "GGA": 4, "TGT": 5}
    dom_size = 3 + 5 * CODON_SIZE
    genome = ("AGACAAAAACTGTGTACTCCGCGATAGACTAGACG" "AGACTATAGCTAGAAGCCCCTGTACTCCGTGTCGATAGACG"
              "AGACTAGGGCCGGGACTGCCGCGACTAGAAGCTAGACTAACG" "AAACCGGGATGTCTGTAT" "CCCCCGGGACTGCCGCGAGGGACTCTGCCGGGAATC")
    res = _lib.extract_domains(genome, [(0, 35, True), (136, 172, True)], dom_size, 3, dom_type_map, one, two)
    assert res[0][0][0] == ((1, 2, 5, 1, 3), 6, 6 + dom_size)
    assert [d[0] for d in res[1][0]] == [(3, 3, 4, 2, 3), (2, 1, 2, 3, 4)]


def test_lib_translate_matches_genetics():
    g = ms.Genetics()
    genomes = [ms.random_genome(800) for _ in range(20)]
    res = _lib.translate_genomes(genomes, g.start_codons, g.stop_codons, g.domain_map, g.one_codon_map,
                                 g.two_codon_map, g.dom_size, g.dom_type_size)
    assert res == g.translate_genomes(genomes)


def test_lib_world_geometry():
    assert _lib.dist_1d(1, 9, 10) == 2
    assert set(_lib.free_moores_nghbhd(0, 0, [(1, 1), (4, 0)], 5)) == {(4, 4), (4, 1), (0, 4), (0, 1), (1, 4), (1, 0)}
    pos = [(0, 0), (1, 1), (3, 3), (4, 4)]
    assert sorted(_lib.get_neighbors([0, 1, 2, 3], [0, 1, 2, 3], pos, 5)) == [(0, 1), (0, 3), (2, 3)]
    parents, children, cpos = _lib.divide_cells_if_possible([0, 2], pos, 4, 5)
    assert parents == [0, 2] and children == [4, 5]
    occupied = set(pos)
    for (x, y), p in zip(cpos, parents):
        assert (x, y) not in occupied and max(_lib.dist_1d(x, pos[p][0], 5), _lib.dist_1d(y, pos[p][1], 5)) == 1
        occupied.add((x, y))
    npos, moved = _lib.move_cells([1], pos, 5)
    assert moved == [1] and npos[0] not in set(pos)


def test_lib_mutations_shapes():
    seqs = [ms.random_genome(500) for _ in range(50)]
    res = _lib.point_mutations(seqs, 1e-2, 0.4, 0.66)
    assert res and all(0 <= i < 50 for _, i in res)
    pairs = list(zip(seqs[:25], seqs[25:]))
    for a, b, i in _lib.recombinations(pairs, 1e-2):
        assert len(a) + len(b) == len(pairs[i][0]) + len(pairs[i][1])


def test_lib_get_proteome_matches_kinetics():
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    w = ms.World(chemistry=CHEMISTRY, map_size=8)
    kin = w.kinetics
    proteome = []
    while not proteome:
        proteome = w.genetics.translate_genomes([ms.random_genome(1500)])[0]
    n_dom = [len(doms) for doms, *_ in proteome]
    per = {"vmaxs": [], "kms": [], "hills": [], "signs": [], "reacts": [], "trnspts": [], "effectors": []}
    for doms, *_ in proteome:
        v = {k: [] for k in per}
        for (t, i0, i1, i2, i3), _, _ in doms:
            v["vmaxs"].append(float(kin.vmax_map.weights[i0 if t != 3 else 0]))
            v["kms"].append(float(kin.km_map.weights[i1]))
            v["hills"].append(int(kin.hill_map.numbers[i0 if t == 3 else 0]))
            v["signs"].append(int(kin.sign_map.signs[i2]))
            v["reacts"].append(kin.reaction_map.M[i3 if t == 1 else 0].tolist())
            v["trnspts"].append(kin.transport_map.M[i3 if t == 2 else 0].tolist())
            v["effectors"].append(kin.effector_map.M[i3 if t == 3 else 0].tolist())
        for k in per:
            per[k].append(v[k])
    dicts = _lib.get_proteome(proteome, molecules=list(kin.mol_names), **per)
    assert [len(d["domains"]) for d in dicts] == n_dom
    got = [ms.Protein.from_dict(d) for d in dicts]
    want = kin.get_proteome(proteome)
    assert [str(p) for p in got] == [str(p) for p in want]
    assert [p.to_dict() for p in got] == [p.to_dict() for p in want]
