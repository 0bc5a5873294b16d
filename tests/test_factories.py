"""Genome factories (reference tests/fast/test_factories.py behaviours)."""
import pytest

import magicsoup_amd as ms
from magicsoup_amd.constants import CODON_SIZE

_X = ms.Molecule("FTx", 10e3)
_Y = ms.Molecule("FTy", 20e3)
_Z = ms.Molecule("FTz", 30e3)


def _world(reactions=()):
    chem = ms.Chemistry(molecules=[_X, _Y, _Z], reactions=list(reactions))
    return ms.World(chemistry=chem, map_size=32)


@pytest.mark.parametrize("size", [0, 7, 250])
def test_empty_proteome_gives_random_filler(size):
    w = _world()
    g = ms.GenomeFact(world=w, proteome=[], target_size=size).generate()
    assert len(g) == size and set(g) <= set("TCGA")
    assert ms.GenomeFact(world=w, proteome=[]).generate() == ""


def test_genome_sizes():
    w = _world([([_X], [_Y]), ([_X, _Y], [_Z])])
    prot = [ms.CatalyticDomainFact(reaction=([_X], [_Y])), ms.TransporterDomainFact(molecule=_Z)]
    with pytest.raises(ValueError):
        ms.GenomeFact(world=w, proteome=[prot], target_size=20)
    assert len(ms.GenomeFact(world=w, proteome=[prot], target_size=300).generate()) == 300
    # start + n domains + stop without filler
    minimal = ms.GenomeFact(world=w, proteome=[prot]).generate()
    assert len(minimal) == 2 * CODON_SIZE + len(prot) * w.genetics.dom_size


def _has(proteome, kind, check):
    return any(isinstance(d, kind) and check(d) for p in proteome for d in p.domains)


def test_generated_genomes_encode_the_proteome():
    w = _world([([_X], [_Y]), ([_X, _Y], [_Z])])
    p0 = [ms.CatalyticDomainFact(reaction=([_X], [_Y])), ms.CatalyticDomainFact(reaction=([_Z], [_X, _Y]))]
    p1 = [ms.TransporterDomainFact(molecule=_X), ms.RegulatoryDomainFact(effector=_Z, is_transmembrane=True, hill=3)]
    fact = ms.GenomeFact(world=w, proteome=[p0, p1], target_size=150)
    hits = 0
    for _ in range(40):  # token codons may randomly contain a stop codon: retry a few times
        g = fact.generate()
        assert len(g) == 150
        w.kill_cells()
        w.spawn_cells([g])
        prots = w.get_cell(by_idx=0).proteome
        ok = (
            _has(prots, ms.CatalyticDomain, lambda d: d.substrates == [_X] and d.products == [_Y])
            and _has(prots, ms.CatalyticDomain, lambda d: d.substrates == [_Z] and d.products == [_X, _Y])
            and _has(prots, ms.TransporterDomain, lambda d: d.molecule is _X)
            and _has(prots, ms.RegulatoryDomain, lambda d: d.effector is _Z and d.hill == 3 and d.is_transmembrane)
        )
        hits += ok
    assert hits >= 3


def test_specified_parameters_are_encoded():
    w = _world([([_X], [_Y])])
    km = 2.0
    fact = ms.GenomeFact(world=w, proteome=[[ms.CatalyticDomainFact(reaction=([_X], [_Y]), km=km, vmax=1.0)]])
    w.spawn_cells([fact.generate() for _ in range(6)])
    doms = [d for i in range(w.n_cells) for p in w.get_cell(by_idx=i).proteome for d in p.domains]
    assert doms
    # the closest representable Km / Vmax of the kinetics maps are chosen
    kms = sorted(set(round(d.km, 6) for d in doms))
    assert len(kms) == 1 and abs(kms[0] - km) / km < 0.5


def test_reaction_orientation_and_unknown_reactions():
    w = _world([([_Y, _X], [_Z])])
    # either orientation of a defined reaction is fine
    ms.GenomeFact(world=w, proteome=[[ms.CatalyticDomainFact(reaction=([_Y, _X], [_Z]))]], target_size=100)
    ms.GenomeFact(world=w, proteome=[[ms.CatalyticDomainFact(reaction=([_Z], [_X, _Y]))]], target_size=100)
    with pytest.raises(ValueError):
        ms.GenomeFact(world=w, proteome=[[ms.CatalyticDomainFact(reaction=([_Y], [_Z]))]], target_size=100)


def test_factories_from_container_dicts():
    w = _world([([_X], [_Y])])
    doms = [
        {"type": "C", "spec": {"reaction": (["FTx"], ["FTy"]), "km": 1.0, "vmax": 2.0}},
        {"type": "T", "spec": {"molecule": "FTz", "is_exporter": True}},
        {"type": "R", "spec": {"effector": "FTy", "hill": 2, "is_inhibiting": False}},
    ]
    facts = [ms.CatalyticDomainFact.from_dict(doms[0]), ms.TransporterDomainFact.from_dict(doms[1]),
             ms.RegulatoryDomainFact.from_dict(doms[2])]
    assert (facts[0].substrates, facts[0].products) == ([_X], [_Y])
    assert facts[1].molecule is _Z and facts[2].hill == 2
    assert len(ms.GenomeFact(world=w, proteome=[facts]).generate()) == 2 * CODON_SIZE + 3 * w.genetics.dom_size
    # whole proteins as written by Protein.to_dict()
    fact = ms.GenomeFact.from_dicts([{"cds_start": 0, "cds_end": 0, "is_fwd": True, "domains": doms}], world=w)
    assert len(fact.generate()) == 2 * CODON_SIZE + 3 * w.genetics.dom_size
