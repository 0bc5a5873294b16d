"""Debug: decomposed speculative activity vs host confirmation, with / without forced rebuilds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import genome_pipeline  # noqa: E402
from magicsoup_amd.parallel import DistributedWorld  # noqa: E402
from magicsoup_amd.parallel import dist_world as dwm  # noqa: E402
from tests.conftest import gen_genomes  # noqa: E402

ms.set_seed(8)
torch.manual_seed(8)
w = ms.World(chemistry=CHEMISTRY, map_size=64, seed=8, device="cpu")
w.spawn_cells(gen_genomes(900, 300))
atp = CHEMISTRY.molname_2_idx["ATP"]


def run(spec, dcap, steps, ops):
    genome_pipeline.D_CAP = dcap
    dwm._DIST_SPECULATE = spec
    dw = DistributedWorld(chemistry=CHEMISTRY, map_size=64, seed=9, device="cuda", strips=True)
    dw.adopt_maps(w)
    dw.scatter_from(w, maps=False)
    ms.set_seed(21)
    torch.manual_seed(21)
    trace = []
    for _ in range(steps):
        dw.enzymatic_activity()
        trace.append(("act", float(dw.cell_molecules.sum())))
        if "kill" in ops:
            dw.kill_cells(dw.cell_molecules[:, atp] < 0.3)
        if "div" in ops:
            dw.divide_cells_t(dw.cell_molecules[:, atp] > 3.0)
        trace.append(("n", dw.n_cells))
        if "rec" in ops:
            dw.recombinate_cells(p=1e-4)
        if "mut" in ops:
            dw.mutate_cells(p=1e-3)
        dw.degrade_molecules()
        dw.diffuse_molecules()
        trace.append(("g", hash(tuple(dw.cell_genomes))))
    dw.enzymatic_activity()
    torch.cuda.synchronize()
    trace.append(("end", float(dw.cell_molecules.sum())))
    dw.close()
    return trace


def dig(dw, tag):
    torch.cuda.synchronize()
    cm = dw.cell_molecules
    pos = dw.cell_positions.long()
    return (tag, dw.n_cells, float(cm.double().sum()), int((pos[:, 0] * 100003 + pos[:, 1]).sum()),
            hash(tuple(dw.cell_genomes)), float(dw.owned_molecule_map().double().sum()))


def run2(spec, steps=2):
    genome_pipeline.D_CAP = 12
    dwm._DIST_SPECULATE = spec
    dw = DistributedWorld(chemistry=CHEMISTRY, map_size=64, seed=9, device="cuda", strips=True)
    dw.adopt_maps(w)
    dw.scatter_from(w, maps=False)
    ms.set_seed(21)
    torch.manual_seed(21)
    tr = []
    for i in range(steps):
        dw.enzymatic_activity(); tr.append(dig(dw, f"{i} act"))
        dw.kill_cells(dw.cell_molecules[:, atp] < 0.3); tr.append(dig(dw, f"{i} kill"))
        dw.divide_cells_t(dw.cell_molecules[:, atp] > 3.0); tr.append(dig(dw, f"{i} div"))
        dw.recombinate_cells(p=1e-4); tr.append(dig(dw, f"{i} rec"))
        dw.mutate_cells(p=1e-3); tr.append(dig(dw, f"{i} mut"))
    dw.close()
    return tr


a2, b2 = run2(True), run2(False)
for x, y in zip(a2, b2):
    print("same" if x == y else "DIFF", x, y if x != y else "", flush=True)

for ops in (("kill", "div", "rec", "mut"), ("div", "rec"), ("div", "mut"), ("kill", "div", "rec")):
    for dcap in (12,):
        a = run(True, dcap, 4, ops)
        b = run(False, dcap, 4, ops)
        first = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), None)
        print(ops, "dcap", dcap, "equal" if first is None else f"first diff at {first}: {a[first]} vs {b[first]}",
              flush=True)
genome_pipeline.D_CAP = 12
