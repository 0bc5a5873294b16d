"""Per-part times of performance/check.py's list-API ``mutations`` benchmark (point_mutations,
get_neighbors, pair list, recombinations) on the given device."""
import sys
import time
from argparse import ArgumentParser

import torch

sys.path.insert(0, "performance")
import check  # noqa: E402

import magicsoup_amd as ms  # noqa: E402


def main() -> None:
    ap = ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    w = ms.World(chemistry=check.CHEMISTRY, device=a.device)
    w.spawn_cells(genomes=check._genomes(10000, 1000))
    genomes = list(w.cell_genomes)
    for _ in range(a.reps):
        t0 = time.perf_counter()
        ms.point_mutations(seqs=genomes)
        t1 = time.perf_counter()
        pairs = w.get_neighbors(cell_idxs=list(range(w.n_cells)))
        t2 = time.perf_counter()
        sp = [(genomes[x], genomes[y]) for x, y in pairs]
        t3 = time.perf_counter()
        ms.recombinations(seq_pairs=sp)
        t4 = time.perf_counter()
        print(f"point_mutations {1e3 * (t1 - t0):7.2f} ms  get_neighbors {1e3 * (t2 - t1):7.2f} ms ({len(pairs)} pairs)"
              f"  pair list {1e3 * (t3 - t2):6.2f} ms  recombinations {1e3 * (t4 - t3):7.2f} ms"
              f"  total {1e3 * (t4 - t0):7.2f} ms", flush=True)


if __name__ == "__main__":
    main()
