"""Kernels of the timed steps of a rocprofv3 kernel trace of bench.py, steps delimited by the
diffusion stencil (one launch per step): wall / busy / launches per step, and the launch sequence
of the step with the median wall time: hardware queue, start / end relative to the previous
stencil's end, and the idle gap of that queue before each kernel (side-stream work shows up on its
own queue).

usage: python scripts/lab/step_kernels.py <kernel_trace.csv> <steps>"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# step marker: the stencil (one launch per step), or with MARKER=<prefix> another once-per-step kernel
# (a strip world splits its stencil into interior + boundary launches: use msd::diffuse_corr_kernel)
import os  # noqa: E402

marker = os.environ.get("MARKER", "void msd::diffuse_stencil4")
marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(marker)]
nst = int(sys.argv[2])
a, b = marks[-nst - 1], marks[-1]
sel = rows[a + 1 : b + 1]
t0 = int(rows[a]["End_Timestamp"])
t1 = int(rows[b]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel)
print(f"{nst} steps: {(t1 - t0) / 1e3 / nst:.1f} us/step wall, {busy / 1e3 / nst:.1f} us busy, "
      f"{len(sel) / nst:.1f} launches/step")
walls = []
for j in range(len(marks) - nst, len(marks)):
    walls.append((int(rows[marks[j]]["End_Timestamp"]) - int(rows[marks[j - 1]]["End_Timestamp"]), j))
med = sorted(walls)[len(walls) // 2]
if os.environ.get("STEP") == "max":  # list the slowest step instead
    med = max(walls)
elif os.environ.get("STEP", "").lstrip("-").isdigit():  # or the k-th timed step (0: the first)
    med = walls[int(os.environ["STEP"])]
print(f"step walls (us): median {statistics.median(w for w, _ in walls) / 1e3:.1f}, "
      f"min {min(walls)[0] / 1e3:.1f}, max {max(walls)[0] / 1e3:.1f}; listing the {os.environ.get('STEP', 'median')} step")
j = med[1]
one = rows[marks[j - 1] + 1 : marks[j] + 1]
base = int(rows[marks[j - 1]]["End_Timestamp"])
# per queue over the timed steps: median (first start, last end, busy) relative to the step start
per_q = {}
for jj in range(len(marks) - nst, len(marks)):
    b0 = int(rows[marks[jj - 1]]["End_Timestamp"])
    qs = {}
    for r in rows[marks[jj - 1] + 1 : marks[jj] + 1]:
        s, e = int(r["Start_Timestamp"]) - b0, int(r["End_Timestamp"]) - b0
        f, l, bz = qs.get(r.get("Queue_Id", "?"), (s, e, 0))
        qs[r.get("Queue_Id", "?")] = (min(f, s), max(l, e), bz + e - s)
    for q, v in qs.items():
        per_q.setdefault(q, []).append(v)
for q, vs in sorted(per_q.items()):
    med3 = [statistics.median(v[i] for v in vs) / 1e3 for i in range(3)]
    print(f"queue {q}: median first start {med3[0]:8.1f}, last end {med3[1]:8.1f}, busy {med3[2]:7.1f} us "
          f"({len(vs)} steps)")
last = {}
for r in one:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get("Queue_Id", "?")
    gap = (s - last.get(q, base)) / 1e3
    last[q] = e
    print(f"q{q:>2} {(s - base) / 1e3:8.1f} {(e - base) / 1e3:8.1f}  gap {gap:6.1f}  dur {(e - s) / 1e3:6.1f}  "
          f"{r['Kernel_Name'][:80]}")
