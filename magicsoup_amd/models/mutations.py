"""Point mutations and recombinations of genome strings (public API).

Behaviour follows the reference ``python/magicsoup/mutations.py:4-51`` / ``rust/mutations.rs``:

* ``point_mutations``: per sequence n ~ Poisson(p * len) distinct positions; each is an indel with
  chance ``p_indel`` (a deletion with chance ``p_del``, else an insertion) or else a substitution
  by a random nucleotide (which may equal the old one). Only mutated sequences are returned, with
  their index.
* ``recombinations``: per pair k ~ Poisson(p * (n0 + n1)) strand breaks over both sequences; the
  pieces are shuffled and re-joined into two sequences of the same total length.

Both run in the OpenMP host core with counter-derived per-item RNG streams (reproducible under
``magicsoup_amd.set_seed``). Worlds on the GPU mutate their device genome arena with the HIP
kernels instead (see ``World.mutate_cells``).
"""
from magicsoup_amd.ops import native


def point_mutations(
    seqs: list[str], p: float = 1e-6, p_indel: float = 0.4, p_del: float = 0.66
) -> list[tuple[str, int]]:
    """Mutated copies ``(sequence, index)`` of the sequences that drew at least one mutation."""
    return native.host().point_mutations(list(seqs), float(p), float(p_indel), float(p_del))


def recombinations(seq_pairs: list[tuple[str, str]], p: float = 1e-7) -> list[tuple[str, str, int]]:
    """Recombined pairs ``(new0, new1, index)`` for the pairs that drew at least one strand break."""
    if len(seq_pairs) == 0:
        return []
    return native.host().recombinations([tuple(d) for d in seq_pairs], float(p))
