"""The timed step of a rocprofv3 kernel trace of bench.py that holds the largest top-up spawn
(``spawn_place_kernel``): every kernel of that step with its queue, start / end relative to the
previous stencil's end and its duration, plus the same totals for the median step, so the spawn's
device cost can be read off the trace.

usage: python scripts/lab/spawn_step.py <kernel_trace.csv>"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void msd::diffuse_stencil4")]
steps = [(marks[j - 1], marks[j]) for j in range(1, len(marks))]


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def wall(a, b):
    return (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e3


spawn = [(a, b) for a, b in steps if any("spawn_place" in r["Kernel_Name"] for r in rows[a + 1 : b + 1])]
med = statistics.median(wall(a, b) for a, b in steps)
print(f"{len(steps)} steps, median wall {med:.1f} us; steps with a spawn: {len(spawn)}")
for a, b in spawn:
    t0 = int(rows[a]["End_Timestamp"])
    sel = rows[a + 1 : b + 1]
    print(f"\nspawn step: wall {wall(a, b):.1f} us, {len(sel)} launches, busy {sum(dur(r) for r in sel):.1f} us")
    for r in sel:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"  q{r.get('Queue_Id', '?'):>3} {s:8.1f} {e:8.1f} dur {dur(r):7.1f}  {r['Kernel_Name'][:90]}")
