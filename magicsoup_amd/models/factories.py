"""Genome factories: generate nucleotide sequences that encode a desired proteome.

Semantics follow the reference ``python/magicsoup/factories.py``:

* each domain factory validates itself against a world's chemistry and emits
  ``dom_type_seq + i0 + i1 + i2 + i3`` (the 2-codon prefix, three 1-codon tokens and a 2-codon token),
  choosing tokens through the Kinetics inverse maps; unspecified values are random non-stop codons;
* ``GenomeFact`` lays proteins out as ``pad + start + domains + stop`` with pads free of start/stop
  codons, so the requested CDSs appear in frame on the forward strand.

Fix relative to the reference: ``GenomeFact.from_dicts`` actually keeps the proteins it parses (the
reference drops them, ``factories.py:487-498``).
"""
from __future__ import annotations

import random
from collections import Counter
from typing import Protocol

from magicsoup_amd.constants import CODON_SIZE
from magicsoup_amd.models.containers import Molecule
from magicsoup_amd.models.world import World
from magicsoup_amd.utils.util import closest_value, random_genome, round_down


class DomainFactType(Protocol):
    """Protocol of domain factories."""

    def validate(self, world: World):
        ...

    def gen_coding_sequence(self, world: World) -> str:
        ...

    @classmethod
    def from_dict(cls, dct: dict) -> "DomainFactType":
        ...


def _codon_for(world: World, value_2_idxs: dict, value) -> str:
    """A codon whose token maps to the available value closest to ``value``."""
    v = closest_value(values=value_2_idxs, key=value)
    return world.genetics.idx_2_one_codon[random.choice(value_2_idxs[v])]


def _random_codon(world: World) -> str:
    return random_genome(s=CODON_SIZE, excl=world.genetics.stop_codons)


def _fmt_opt(parts: list[str], km, vmax=None) -> list[str]:
    if km is not None:
        parts.append(f"Km={km:.2e}")
    if vmax is not None:
        parts.append(f"Vmax={vmax:.2e}")
    return parts


class CatalyticDomainFact:
    """Factory for catalytic domain sequences.

    Arguments:
        reaction: ``(substrates, products)`` of a reaction of the world's chemistry (either
            direction).
        km / vmax: Desired Km (mM) / Vmax (mmol/s); the closest available value is used, random if
            ``None``.
    """

    def __init__(self, reaction: tuple[list[Molecule], list[Molecule]], km: float | None = None, vmax: float | None = None):
        subs, prods = reaction
        self.substrates = sorted(subs)
        self.products = sorted(prods)
        self.km = km
        self.vmax = vmax

    def validate(self, world: World):
        known = set()
        for s, p in world.chemistry.reactions:
            known.add((tuple(sorted(s)), tuple(sorted(p))))
            known.add((tuple(sorted(p)), tuple(sorted(s))))
        if (tuple(self.substrates), tuple(self.products)) not in known:
            lft = " + ".join(d.name for d in self.substrates)
            rgt = " + ".join(d.name for d in self.products)
            raise ValueError(
                f"CatalyticDomainFact has this reaction defined: {lft} <-> {rgt}."
                " This world's chemistry doesn't define this reaction."
            )

    def gen_coding_sequence(self, world: World) -> str:
        kin, gen = world.kinetics, world.genetics
        seq = random.choice(gen.domain_types[1])
        seq += _codon_for(world, kin.vmax_2_idxs, self.vmax) if self.vmax is not None else _random_codon(world)
        seq += _codon_for(world, kin.km_2_idxs, self.km) if self.km is not None else _random_codon(world)
        react = (tuple(self.substrates), tuple(self.products))
        is_fwd = react in kin.catal_2_idxs
        if not is_fwd:
            react = (tuple(self.products), tuple(self.substrates))
        seq += gen.idx_2_one_codon[random.choice(kin.sign_2_idxs[is_fwd])]
        seq += gen.idx_2_two_codon[random.choice(kin.catal_2_idxs[react])]
        return seq

    @classmethod
    def from_dict(cls, dct: dict) -> "CatalyticDomainFact":
        spec = dct["spec"]
        lft, rgt = spec["reaction"]
        reaction = ([Molecule.from_name(d) for d in lft], [Molecule.from_name(d) for d in rgt])
        return cls(reaction=reaction, km=spec.get("km"), vmax=spec.get("vmax"))

    def __repr__(self) -> str:
        ins = ",".join(str(d) for d in self.substrates)
        outs = ",".join(str(d) for d in self.products)
        return f"CatalyticDomain({','.join(_fmt_opt([f'{ins}<->{outs}'], self.km, self.vmax))})"

    def __str__(self) -> str:
        def cnt(ms):
            return " + ".join(f"{n} {k}" for k, n in Counter(str(d) for d in ms).items())

        out = f"{cnt(self.substrates)} <-> {cnt(self.products)}"
        opt = [f"Km {self.km:.2e}"] if self.km is not None else []
        opt += [f"Vmax {self.vmax:.2e}"] if self.vmax is not None else []
        return out if not opt else out + " | " + " ".join(opt)


class TransporterDomainFact:
    """Factory for transporter domain sequences of ``molecule`` (optionally with Km, Vmax and
    direction)."""

    def __init__(self, molecule: Molecule, km: float | None = None, vmax: float | None = None, is_exporter: bool | None = None):
        self.molecule = molecule
        self.km = km
        self.vmax = vmax
        self.is_exporter = is_exporter

    def validate(self, world: World):
        if self.molecule not in world.chemistry.molecules:
            raise ValueError(
                f"TransporterDomainFact has this molecule defined: {self.molecule}."
                " This world's chemistry doesn't define this molecule species."
            )

    def gen_coding_sequence(self, world: World) -> str:
        kin, gen = world.kinetics, world.genetics
        seq = random.choice(gen.domain_types[2])
        seq += _codon_for(world, kin.vmax_2_idxs, self.vmax) if self.vmax is not None else _random_codon(world)
        seq += _codon_for(world, kin.km_2_idxs, self.km) if self.km is not None else _random_codon(world)
        if self.is_exporter is not None:
            seq += gen.idx_2_one_codon[random.choice(kin.sign_2_idxs[self.is_exporter])]
        else:
            seq += _random_codon(world)
        seq += gen.idx_2_two_codon[random.choice(kin.trnsp_2_idxs[self.molecule])]
        return seq

    @classmethod
    def from_dict(cls, dct: dict) -> "TransporterDomainFact":
        spec = dct["spec"]
        return cls(
            molecule=Molecule.from_name(spec["molecule"]),
            km=spec.get("km"),
            vmax=spec.get("vmax"),
            is_exporter=spec.get("is_exporter"),
        )

    def __repr__(self) -> str:
        parts = _fmt_opt([str(self.molecule)], self.km, self.vmax)
        if self.is_exporter is not None:
            parts.append("exporter" if self.is_exporter else "importer")
        return f"TransporterDomain({','.join(parts)})"

    def __str__(self) -> str:
        kind = "transporter" if self.is_exporter is None else ("exporter" if self.is_exporter else "importer")
        opt = [f"Km {self.km:.2e}"] if self.km is not None else []
        opt += [f"Vmax {self.vmax:.2e}"] if self.vmax is not None else []
        out = f"{self.molecule} {kind}"
        return out if not opt else out + " | " + " ".join(opt)


class RegulatoryDomainFact:
    """Factory for regulatory domain sequences sensing ``effector`` (intracellular, or
    extracellular if ``is_transmembrane``); Hill coefficients 1, 3 and 5 are available."""

    def __init__(
        self,
        effector: Molecule,
        is_transmembrane: bool,
        is_inhibiting: bool | None = None,
        km: float | None = None,
        hill: int | None = None,
    ):
        self.effector = effector
        self.is_transmembrane = is_transmembrane
        self.is_inhibiting = is_inhibiting
        self.km = km
        self.hill = hill

    def validate(self, world: World):
        if self.effector not in world.chemistry.molecules:
            raise ValueError(
                f"RegulatoryDomainFact has this effector defined: {self.effector}."
                " This world's chemistry doesn't define this molecule species."
            )

    def gen_coding_sequence(self, world: World) -> str:
        kin, gen = world.kinetics, world.genetics
        seq = random.choice(gen.domain_types[3])
        if self.hill is not None:
            h = int(closest_value(values=kin.hill_2_idxs, key=self.hill))
            seq += gen.idx_2_one_codon[random.choice(kin.hill_2_idxs[h])]
        else:
            seq += _random_codon(world)
        seq += _codon_for(world, kin.km_2_idxs, self.km) if self.km is not None else _random_codon(world)
        if self.is_inhibiting is not None:
            seq += gen.idx_2_one_codon[random.choice(kin.sign_2_idxs[not self.is_inhibiting])]
        else:
            seq += _random_codon(world)
        seq += gen.idx_2_two_codon[random.choice(kin.regul_2_idxs[(self.effector, self.is_transmembrane)])]
        return seq

    @classmethod
    def from_dict(cls, dct: dict) -> "RegulatoryDomainFact":
        spec = dct["spec"]
        return cls(
            effector=Molecule.from_name(spec["effector"]),
            km=spec.get("km"),
            hill=spec.get("hill"),
            is_inhibiting=spec.get("is_inhibiting"),
            is_transmembrane=bool(spec.get("is_transmembrane", False)),
        )

    def __repr__(self) -> str:
        parts = _fmt_opt([f"{self.effector}"], self.km)
        if self.hill is not None:
            parts.append(f"hill={self.hill}")
        parts.append("transmembrane" if self.is_transmembrane else "cytosolic")
        if self.is_inhibiting is not None:
            parts.append("inhibiting" if self.is_inhibiting else "activating")
        return f"ReceptorDomain({','.join(parts)})"

    def __str__(self) -> str:
        loc = "[e]" if self.is_transmembrane else "[i]"
        eff = "effector" if self.is_inhibiting is None else (" inhibitor" if self.is_inhibiting else " activator")
        opt = [f"Km {self.km:.2e}"] if self.km is not None else []
        opt += [f"Hill {self.hill}"] if self.hill is not None else []
        out = f"{self.effector}{loc} {eff}"
        return out if not opt else out + " | " + " ".join(opt)


_FACTS = {"C": CatalyticDomainFact, "T": TransporterDomainFact, "R": RegulatoryDomainFact}


class GenomeFact:
    """Generate genomes that encode ``proteome`` (a list of proteins, each a list of domain
    factories) in one reading frame of the forward strand.

    Arguments:
        world: World whose genetics / kinetics maps are used.
        proteome: list of lists of domain factories.
        target_size: Genome length; the minimum ``sum(dom_size * n_domains + 6)`` if ``None``.
            Padding between proteins contains no start or stop codons.
    """

    def __init__(self, world: World, proteome: list[list[DomainFactType]], target_size: int | None = None):
        self.world = world
        self.proteome = proteome
        try:
            prots = list(proteome)
        except TypeError as err:
            raise ValueError("Proteome must be a list of lists representing domains in proteins.") from err
        for pi, prot in enumerate(prots):
            try:
                iter(prot)
            except TypeError as err:
                raise ValueError(
                    "Proteome must be a list of lists representing domains in proteins."
                    f" Element {pi} of proteome is not iterable."
                ) from err
        for prot in prots:
            for dom in prot:
                dom.validate(world=world)
        self.req_nts = sum(world.genetics.dom_size * len(p) + 2 * CODON_SIZE for p in prots)
        self.target_size = self.req_nts if target_size is None else target_size
        if self.req_nts > self.target_size:
            raise ValueError(
                "Genome size too small."
                f" The given proteome would require at least {self.req_nts} nucleotides."
                f" But the given genome target size is target_size={self.target_size}."
            )

    def generate(self) -> str:
        """A new random genome encoding the proteome."""
        gen = self.world.genetics
        cdss = ["".join(d.gen_coding_sequence(world=self.world) for d in p) for p in self.proteome]
        n_pads = len(cdss) + 1
        free = self.target_size - self.req_nts
        pad = round_down(free / n_pads, to=1)
        excl = gen.start_codons + gen.stop_codons
        pads = [random_genome(s=pad, excl=excl) for _ in range(n_pads)]
        tail = random_genome(s=free - n_pads * pad, excl=excl)
        parts: list[str] = []
        for cds in cdss:
            parts += [pads.pop(), random.choice(gen.start_codons), cds, random.choice(gen.stop_codons)]
        parts += [pads.pop(), tail]
        return "".join(parts)

    @classmethod
    def from_dicts(cls, dcts: list[dict], world: World) -> "GenomeFact":
        """Factory from ``Protein.to_dict()`` representations."""
        prots = [[_FACTS[d["type"]].from_dict(d) for d in p["domains"] if d["type"] in _FACTS] for p in dcts]
        return GenomeFact(proteome=prots, world=world)
