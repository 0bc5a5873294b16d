"""Log every capacity reallocation of the per-cell stores during bench steps (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from magicsoup_amd.models import kinetics as K  # noqa: E402
from magicsoup_amd.models import strings as S  # noqa: E402
from magicsoup_amd.models import world as W  # noqa: E402

log = []


def wrap(cls, name, tag, probe):
    orig = getattr(cls, name)

    def f(self, *a, **kw):
        before = probe(self)
        out = orig(self, *a, **kw)
        after = probe(self)
        if before != after:
            log.append((tag, before, after))
        return out

    setattr(cls, name, f)


wrap(S.StringArena, "reserve", "arena.reserve", lambda s: (s.data.data_ptr(), tuple(s.data.shape)))
def _kcap(s):
    b = s.__dict__.get("_bufs", {}).get("N")
    return (0, 0) if b is None else (b.data_ptr(), b.size(0))


wrap(K.Kinetics, "increase_max_cells", "kin.grow_cells", _kcap)
wrap(K.Kinetics, "_commit_compact", "kin.compact", _kcap)
wrap(K.Kinetics, "increase_max_proteins", "kin.grow_prot", lambda s: tuple(s.N.shape))
wrap(W._Column, "reserve", "col.reserve", lambda s: (s.buf.data_ptr(), tuple(s.buf.shape)))


def main():
    import magicsoup_amd as ms
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY

    dev = "cuda"
    w = ms.World(chemistry=CHEMISTRY, map_size=4096, device=dev, seed=0)
    w.spawn_cells(bench.random_genomes(50_000, 500, dev))
    atp = CHEMISTRY.molname_2_idx["ATP"]
    for i in range(15):
        log.clear()
        bench.step(w, 50_000, 500, atp)
        torch.cuda.synchronize()
        g = w._genomes
        print(f"step {i}: n={w.n_cells} P={w.kinetics.N.size(1)} arena={tuple(g.data.shape)} "
              f"maxlen={int(g.lens[:g.n].max())} reallocs={[(t, b[-1], a[-1]) for t, b, a in log]}", flush=True)


if __name__ == "__main__":
    main()
