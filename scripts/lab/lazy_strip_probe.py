"""Where a virtual-strip world with lazy divisions departs from the eager protocol: the reference
loop in both modes, with a fingerprint of the state after every op (one rank over RCCL)."""
import os
import random
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def fp(dw):
    n = dw.n_cells
    g = list(dw.cell_genomes)
    return (n, float(dw.cell_molecules.double().sum()), int(dw.cell_divisions.sum()), hash(tuple(g)),
            float(dw.owned_molecule_map().double().sum()), int(dw.cell_map.sum()), float(dw.kinetics.N.double().abs().sum()))


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import magicsoup_amd as ms
    from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY as chem
    from magicsoup_amd.parallel import DistributedWorld
    from tests.conftest import gen_genomes

    ms.set_seed(21)
    torch.manual_seed(21)
    w = ms.World(chemistry=chem, map_size=64, seed=21, device="cpu")
    w.spawn_cells(gen_genomes(1200, 300))
    atp = chem.molname_2_idx["ATP"]
    logs = {}
    from magicsoup_amd.parallel import dist_world as dwm

    genomes = {}
    for mode in ("eager", "eager_xb_late", "lazy", "lazy_resolve_early", "lazy_resolve_at_once"):
        lazy = mode.startswith("lazy")
        dwm._XB_EARLY = mode == "eager"
        random.seed(5)
        dw = DistributedWorld(chemistry=chem, map_size=64, seed=22, device="cuda", strips=True)
        dw.adopt_maps(w)
        dw.scatter_from(w, maps=False)
        ms.set_seed(23)
        log = []
        for it in range(4):
            dw.enzymatic_activity()
            log.append((it, "activity", fp(dw)))
            dw.kill_cells(dw.cell_molecules[:, atp] < 0.5)
            log.append((it, "kill", fp(dw)))
            repl = dw.cell_molecules[:, atp] > 2.0
            dw.cell_molecules[:, atp] -= 1.0 * repl
            dw.divide_cells_t(repl, lazy=lazy)
            if mode == "lazy_resolve_at_once":
                dev_st = dw.__dict__["_hip_scratch"].bufs["dv_status"][:20].tolist()
                dw._resolve_count()
                print("host_st", dw.__dict__["_dv_host_st"].tolist(), "dev", dev_st, flush=True)
            dw.recombinate_cells(p=1e-4)
            dw.mutate_cells(p=1e-4)
            if mode == "lazy_resolve_early":
                dw._resolve_count()
            dw.degrade_molecules()
            dw.diffuse_molecules()
            if it == 0:
                genomes[mode] = (list(dw.cell_genomes), dw.n_cells)
            log.append((it, "diffuse", fp(dw), dict(dw.migrated)))
            dw.increment_cell_lifetimes()
        logs[mode] = log
        dw.close()
    ge = genomes["eager_xb_late"][0]
    for other in ("lazy", "lazy_resolve_early", "lazy_resolve_at_once"):
        gl = genomes[other][0]
        bad = [i for i, (x, y) in enumerate(zip(ge, gl)) if x != y]
        print("genome diffs", other, len(bad), bad[:20], [(len(ge[i]), len(gl[i])) for i in bad[:5]], flush=True)
    for other in ("eager_xb_late", "lazy", "lazy_resolve_early", "lazy_resolve_at_once"):
        for a, b in zip(logs["eager"], logs[other]):
            tag = "same" if a[2] == b[2] else "DIFF"
            print(tag, other, a[0], a[1], a[2], b[2], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
