"""Multi-GPU execution over torch.distributed (RCCL over xGMI).

* :class:`DistributedWorld` -- one world domain-decomposed into row strips, one strip per rank
  (halo exchange, cell migration, global reductions).
* :class:`GlobalWorld` -- the reference ``World`` API with global cell indices over a
  DistributedWorld (uniform placement over the whole torus, index semantics of world.py).
* :class:`Ensemble` -- independent replicate worlds, one per rank (no communication in the step).
"""
from magicsoup_amd.parallel.dist_world import DistributedWorld
from magicsoup_amd.parallel.ensemble import Ensemble
from magicsoup_amd.parallel.global_world import GlobalWorld

__all__ = ["DistributedWorld", "Ensemble", "GlobalWorld"]
