"""Untraced host / device timeline of bench steps: every World op call is bracketed by host
timestamps and HIP events recorded on the compute stream (an event completes when the device has
finished all work issued before it), so for each op we see when the host issued it and when the
device reached / finished it -- without a tracer in the loop. Prints the median over steps.

usage: python scripts/lab/step_timeline.py [map_size] [cells] [steps] [pipelined]
    pipelined (any 4th argument): no synchronisation between steps (as in bench.py); device times
    are then relative to the point where the device finished the previous step's work."""
import collections
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import magicsoup_amd as ms  # noqa: E402
from magicsoup_amd.examples.wood_ljungdahl import CHEMISTRY  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50000
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
pipelined = len(sys.argv) > 4
w = ms.World(chemistry=CHEMISTRY, map_size=S, device="cuda", seed=0)
w.spawn_cells(bench.random_genomes(N, 500, "cuda"))
atp = CHEMISTRY.molname_2_idx["ATP"]
for _ in range(20):
    bench.step(w, N, 500, atp)
torch.cuda.synchronize()

names = ("spawn_cells", "enzymatic_activity", "kill_cells", "divide_cells_t", "recombinate_cells", "mutate_cells",
         "degrade_molecules", "diffuse_molecules", "increment_cell_lifetimes")
log = []
cls = type(w)
orig = {nm: getattr(cls, nm) for nm in names}


def make(f, nm):
    def wrap(self, *a, **k):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        e0.record()
        try:
            return f(self, *a, **k)
        finally:
            e1.record()
            log.append((nm, h0, time.perf_counter(), e0, e1))
    return wrap


for nm in names:
    setattr(cls, nm, make(orig[nm], nm))
raw = []
for _ in range(steps):
    log.clear()
    if not pipelined:
        torch.cuda.synchronize()
    z = torch.cuda.Event(enable_timing=True)
    hz = time.perf_counter()
    z.record()
    bench.step(w, N, 500, atp)
    zend = torch.cuda.Event(enable_timing=True)
    zend.record()
    raw.append((list(log), hz, z, zend, time.perf_counter()))
torch.cuda.synchronize()
per_step = []
for lg, hz, z, zend, hend in raw:
    rows = [(nm, (h0 - hz) * 1e6, (h1 - hz) * 1e6, z.elapsed_time(e0) * 1e3, z.elapsed_time(e1) * 1e3)
            for nm, h0, h1, e0, e1 in lg]
    per_step.append((rows, (hend - hz) * 1e6, z.elapsed_time(zend) * 1e3))
for nm, f in orig.items():
    setattr(cls, nm, f)
# steps with the most common op sequence
seqs = collections.Counter(tuple(r[0] for r in rows) for rows, _, _ in per_step)
seq = seqs.most_common(1)[0][0]
sel = [p for p in per_step if tuple(r[0] for r in p[0]) == seq]
print(f"{S}^2 / {N}: {len(sel)} of {steps} steps with the op sequence below; median host issue end "
      f"{statistics.median(p[1] for p in sel):.0f} us, device end {statistics.median(p[2] for p in sel):.0f} us")
print(f"{'op':26s} {'host_in':>8s} {'host_out':>8s} {'dev_in':>8s} {'dev_out':>8s}   (us from step start)")
for i, nm in enumerate(seq):
    vals = [statistics.median(p[0][i][j] for p in sel) for j in range(1, 5)]
    print(f"{nm:26s} {vals[0]:8.0f} {vals[1]:8.0f} {vals[2]:8.0f} {vals[3]:8.0f}")
