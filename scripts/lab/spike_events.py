"""Per-step wall time of pipelined bench steps (an event pair brackets each step, read after the
run) together with the rare internal events that happened in that step (storage growth, row
recycling, parameter re-layouts, spawns, rollbacks, scratch allocations): what makes slow steps slow.

usage: python scripts/lab/spike_events.py [map_size] [cells] [steps] [warmup]"""
import collections
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 80
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 20
_MDT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[os.environ.get("MS_MAP_DTYPE", "fp32")]
events = collections.Counter()
TARGETS = [
    ("magicsoup_amd.models.kinetics", "Kinetics", "_recycle_rows"),
    ("magicsoup_amd.models.kinetics", "Kinetics", "increase_max_proteins"),
    ("magicsoup_amd.models.kinetics", "Kinetics", "_materialize"),
    ("magicsoup_amd.models.kinetics", "Kinetics", "_slot_reserve"),
    ("magicsoup_amd.models.strings", "StringArena", "reserve"),
    ("magicsoup_amd.models.world", "_Column", "reserve"),
    ("magicsoup_amd.models.world", "World", "spawn_cells"),
    ("magicsoup_amd.ops.genome_pipeline", None, "_resolve"),
    ("magicsoup_amd.ops.hip_ops", None, "restore_cell_state"),
    ("magicsoup_amd.models.world", "World", "_update_params_rows"),
]


def wrap(f, key):
    def w(*a, **k):
        out = f(*a, **k)
        if key.endswith("_resolve"):
            if out:
                events["resolve:rebuilt"] += 1
        elif key.endswith(".reserve") or key.endswith("_slot_reserve"):
            pass
        else:
            events[key] += 1
        return out
    return w


def wrap_growth(f, key, size_of):
    def w(self, *a, **k):
        before = size_of(self)
        out = f(self, *a, **k)
        if size_of(self) != before:
            events[key + ":grew"] += 1
        return out
    return w


w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0, map_dtype=_MDT)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(warm):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
sizes = {
    "StringArena.reserve": lambda a: (a.data.data_ptr(), a.width),
    "_Column.reserve": lambda c: c.buf.data_ptr(),
    "Kinetics._slot_reserve": lambda k: (k.__dict__.get("_slot_buf").data_ptr() if k.__dict__.get("_slot_buf") is not None else 0),
}
for mod, cls, fn in TARGETS:
    m = importlib.import_module(mod)
    owner = getattr(m, cls) if cls else m
    key = f"{cls}.{fn}" if cls else f"{mod.split('.')[-1]}.{fn}"
    if key in sizes:
        setattr(owner, fn, wrap_growth(getattr(owner, fn), key, sizes[key]))
    else:
        setattr(owner, fn, wrap(getattr(owner, fn), key))
from magicsoup_amd.ops import hip_ops  # noqa: E402

orig_get = hip_ops.Scratch.get


def get(self, name, numel, dtype, device, zero=False):
    t = self.bufs.get(name)
    if t is None or t.numel() < numel or t.dtype != dtype or t.device != device:
        events[f"scratch:{name}"] += 1
    return orig_get(self, name, numel, dtype, device, zero)


hip_ops.Scratch.get = get
import gc  # noqa: E402
import time  # noqa: E402

_gc_t = {}


def _gc_cb(phase, info):
    if phase == "start":
        _gc_t["t"] = time.perf_counter()
    else:
        events[f"gc{info['generation']}_us"] += int((time.perf_counter() - _gc_t.get("t", time.perf_counter())) * 1e6)


gc.callbacks.append(_gc_cb)
recs = []
for _ in range(steps):
    events.clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    bench.step(w, N, 500, atp)
    e1.record()
    recs.append((e0, e1, dict(events)))
torch.cuda.synchronize()
times = [e0.elapsed_time(e1) for e0, e1, _ in recs]
med = sorted(times)[len(times) // 2]
kin = w.kinetics
print(f"{S}^2 / {N}: {steps} steps, median {med:.3f} ms, mean {sum(times) / len(times):.3f} ms; proteins P={kin._P()}, "
      f"storage rows {min(int(t.size(0)) for t in kin._store.values())}, arena width {w._genomes.width}, "
      f"max genome {int(w._genomes.lens[:w.n_cells].max())}")
for i, ((e0, e1, ev), t) in enumerate(zip(recs, times)):
    if t > 1.25 * med or ev or warm == 0:
        print(f"  step {i:3d} {t:7.3f} ms  {ev}")
