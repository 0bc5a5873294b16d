"""magicsoup_amd — an MI355X-native cell metabolism and evolution simulator.

Drop-in for the reference ``magicsoup`` API (``import magicsoup_amd as ms``; the ``magicsoup``
package in this repository re-exports it under the reference's module paths):

    ms.Molecule, ms.Chemistry, ms.World, ms.Cell, ms.Protein, ms.CatalyticDomain,
    ms.TransporterDomain, ms.RegulatoryDomain, ms.Genetics, ms.Kinetics,
    ms.GenomeFact, ms.CatalyticDomainFact, ms.TransporterDomainFact, ms.RegulatoryDomainFact,
    ms.point_mutations, ms.recombinations, ms.random_genome, ...

Layout: ``models/`` (data model, genetics, kinetics, world, factories), ``ops/`` (native dispatch,
HIP kernels in ``csrc/hip``, OpenMP host core in ``csrc/host``), ``parallel/`` (domain-decomposed
multi-GPU world over RCCL), ``utils/`` (helpers, profiling, checkpointing), ``examples/``
(chemistries).
"""
from magicsoup_amd.constants import CODON_SIZE, GAS_CONSTANT, ALL_NTS, ALL_CODONS, DomainSpecType, ProteinSpecType
from magicsoup_amd.utils.util import (
    round_down,
    closest_value,
    randstr,
    random_genome,
    variants,
    codons,
    dist_1d,
    free_moores_nghbhd,
)
from magicsoup_amd.models.containers import (
    Molecule,
    Chemistry,
    DomainType,
    CatalyticDomain,
    TransporterDomain,
    RegulatoryDomain,
    Protein,
    Cell,
)
from magicsoup_amd.models.mutations import point_mutations, recombinations
from magicsoup_amd.models.genetics import Genetics
from magicsoup_amd.models.kinetics import Kinetics
from magicsoup_amd.models.world import World
from magicsoup_amd.models.factories import (
    DomainFactType,
    CatalyticDomainFact,
    TransporterDomainFact,
    RegulatoryDomainFact,
    GenomeFact,
)
from magicsoup_amd.ops.world_ops import set_seed as _set_seed

__version__ = "0.1.0"


def set_seed(seed: int) -> None:
    """Seed the native RNG streams (placement, mutations, recombinations, labels) on all devices."""
    import random as _random
    import torch as _torch

    _random.seed(seed)
    _set_seed(seed, "cuda" if _torch.cuda.is_available() else None)
