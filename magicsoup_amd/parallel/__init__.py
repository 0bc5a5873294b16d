"""Multi-GPU execution: a domain-decomposed World over torch.distributed (RCCL over xGMI)."""
