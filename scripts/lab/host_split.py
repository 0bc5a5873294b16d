"""Where the host spends a pipelined bench step: per top-level World op, the inclusive host time
split into time BLOCKED in synchronisations (wait_count, guarded waits, tolist / item, stream and
event syncs) and BUSY (issuing work). The busy total is the step's host floor; blocked time is
the device running ahead of the host's need.

usage: python scripts/lab/host_split.py [map_size] [cells] [steps]
MS_VIRTUAL_STRIPS=1: a one-rank DistributedWorld running the strip protocol (RCCL to itself).
MS_NATIVE_TIMES=1 / MS_PY_TIMES=1: host time per native entry point / selected Python helper;
MS_CPROFILE=1: cProfile of the timed steps (inflates the totals; read the ranking)."""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402
from magicsoup_amd.ops import hip_ops  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1448
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6250
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 20

OPS = ["spawn_cells", "enzymatic_activity", "kill_divide_where", "kill_divide_t", "kill_cells", "divide_cells_t", "recombinate_cells", "mutate_cells",
       "degrade_molecules", "diffuse_molecules", "increment_cell_lifetimes"]
busy = collections.defaultdict(float)
blocked = collections.defaultdict(float)
calls = collections.defaultdict(int)
stack = []  # the op being timed (outermost only)
blk = [0.0]  # blocked time accumulated since the op started


def blocking(f):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            blk[0] += time.perf_counter() - t0
    return w


def op(f, name):
    def w(*a, **k):
        if stack:
            return f(*a, **k)
        stack.append(name)
        b0, t0 = blk[0], time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            dt, db = time.perf_counter() - t0, blk[0] - b0
            busy[name] += dt - db
            blocked[name] += db
            calls[name] += 1
            stack.pop()
    return w


hip_ops.wait_count = blocking(hip_ops.wait_count)
hip_ops.guarded_sync = blocking(hip_ops.guarded_sync)
torch.Tensor.tolist = blocking(torch.Tensor.tolist)
torch.Tensor.item = blocking(torch.Tensor.item)
torch.cuda.synchronize = blocking(torch.cuda.synchronize)
torch.cuda.Event.synchronize = blocking(torch.cuda.Event.synchronize)
torch.cuda.Stream.synchronize = blocking(torch.cuda.Stream.synchronize)

# host time inside each native entry point (a proxy module in front of the extension)
native_t = collections.defaultdict(float)
native_n = collections.defaultdict(int)


class _Timed:
    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        f = getattr(self._mod, name)
        if not callable(f) or isinstance(f, type):
            return f

        def w(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                native_t[name] += time.perf_counter() - t0
                native_n[name] += 1
        return w


if os.environ.get("MS_NATIVE_TIMES") == "1":
    from magicsoup_amd.ops import native

    native._mods["_hip"] = _Timed(native.hip())

# MS_PY_TIMES=1: inclusive host time of selected Python helpers (nested calls counted in each)
py_t = collections.defaultdict(float)
py_n = collections.defaultdict(int)


def _timed_py(f, name):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            py_t[name] += time.perf_counter() - t0
            py_n[name] += 1
    return w


if os.environ.get("MS_PY_TIMES") == "1":
    from magicsoup_amd.models import kinetics as kin_mod
    from magicsoup_amd.models import world as world_mod
    from magicsoup_amd.ops import genome_pipeline, streams, world_ops

    targets = [
        (genome_pipeline, ["recombinate_all", "point_mutations", "_begin", "_kin_desc", "_arena_desc", "_gen_desc",
                           "_blob", "_record", "reconcile", "_resolve"]),
        (hip_ops, ["diffuse", "permeate", "enzymatic_activity", "_launch_integrate", "degrade", "neighbor_slot_args",
                   "map_for_pixels", "_rng", "_check_overflow", "cell_state_buffer"]),
        (world_ops, ["diffuse", "permeate", "enzymatic_activity", "fused_activity", "degrade"]),
        (world_mod.World, ["_flush_deferred", "_reconcile", "_fast_world", "_adopt_count", "_defer", "_resolve_count",
                           "_divide_mask_gpu", "_watch_genome_width", "_join_side", "_defer_genome_op"]),
        (kin_mod.Kinetics, ["_kernel_params", "_row_limit", "_reserve_rows", "_enter_slot_mode", "_slot_tensor",
                            "_sync", "_pack_ok"]),
        (streams.NEvent, ["record", "wait", "synchronize", "__init__"]),
        (streams, ["join"]),
    ]
    for obj, names in targets:
        for nm in names:
            f = obj.__dict__.get(nm) if isinstance(obj, type) else getattr(obj, nm, None)
            if f is None:
                continue
            label = f"{getattr(obj, '__name__', '?').split('.')[-1]}.{nm}"
            setattr(obj, nm, _timed_py(f, label))

virtual = os.environ.get("MS_VIRTUAL_STRIPS") == "1"
if virtual:
    import torch.distributed as dist

    from magicsoup_amd.parallel import DistributedWorld

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29547")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    w = DistributedWorld(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0, strips=True)
    cls = DistributedWorld
else:
    w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
    cls = ms.World
for name in OPS:
    for c in (ms.World, cls):
        if name in c.__dict__:
            setattr(c, name, op(c.__dict__[name], name))
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(warm):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
for d in (busy, blocked, calls, native_t, native_n, py_t, py_n):
    d.clear()
blk[0] = 0.0
_hipm = hip_ops._m()
gb0 = _hipm.graph_batch_stats() if hasattr(_hipm, "graph_batch_stats") else None
prof = None
if os.environ.get("MS_CPROFILE") == "1":  # per-function host time (tottime) of the timed steps
    import cProfile

    prof = cProfile.Profile()
    prof.enable()
t0 = time.perf_counter()
for _ in range(steps):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / steps * 1e6
if gb0 is not None:  # graph batching of the native launches (csrc/hip/launch.h), per step
    gb1 = _hipm.graph_batch_stats()
    per = {k: round((gb1[k] - gb0[k]) / steps, 2) for k in ("graph_launches", "graph_nodes", "direct", "updated_nodes",
                                                             "instantiated", "flushes")}
    hist = {int(k): round((v - gb0["batch_sizes"].get(k, 0)) / steps, 2) for k, v in gb1["batch_sizes"].items()}
    print("graph batching per step:", per, "batch lengths:", {k: v for k, v in sorted(hist.items()) if v})
if prof is not None:
    import io
    import pstats

    prof.disable()
    buf = io.StringIO()
    pstats.Stats(prof, stream=buf).sort_stats(os.environ.get("MS_CPROFILE_SORT", "tottime")).print_stats(int(os.environ.get("MS_CPROFILE_N", "45")))
    print(buf.getvalue())
tb, tk = sum(busy.values()) / steps * 1e6, sum(blocked.values()) / steps * 1e6
print(f"{S}^2 / {N}{' virtual' if virtual else ''}: wall {wall:.0f} us/step; inside ops: busy {tb:.0f}, blocked {tk:.0f}; "
      f"outside ops (bench glue) {wall - tb - tk:.0f}")
print(f"  {'op':28s} {'busy us':>8s} {'blocked':>8s} {'calls':>6s}")
for name in sorted(busy, key=lambda k: -busy[k]):
    print(f"  {name:28s} {busy[name] / steps * 1e6:8.1f} {blocked[name] / steps * 1e6:8.1f} {calls[name] / steps:6.2f}")
if native_t:
    print(f"  native entry points: {sum(native_t.values()) / steps * 1e6:.0f} us/step host in {sum(native_n.values()) / steps:.0f} calls")
    for name in sorted(native_t, key=lambda k: -native_t[k])[:40]:
        print(f"    {name:32s} {native_t[name] / steps * 1e6:8.1f} us {native_n[name] / steps:6.2f} calls")
if py_t:
    print("  python helpers (inclusive us/step, calls/step):")
    for name in sorted(py_t, key=lambda k: -py_t[k]):
        print(f"    {name:40s} {py_t[name] / steps * 1e6:8.1f} us {py_n[name] / steps:6.2f} calls")
if virtual:
    w.close()
