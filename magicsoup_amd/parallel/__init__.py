"""Multi-GPU execution: a domain-decomposed World over torch.distributed (RCCL over xGMI)."""
from magicsoup_amd.parallel.dist_world import DistributedWorld

__all__ = ["DistributedWorld"]
