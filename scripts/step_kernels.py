"""Kernels of the timed steps of a rocprofv3 kernel trace of bench.py, steps delimited by the
diffusion stencil (one launch per step): wall / busy / launches per step and one step's launch
sequence with the idle gap before each kernel.

usage: python scripts/step_kernels.py <kernel_trace.csv> <steps>"""
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("void msd::diffuse_stencil4")]
nst = int(sys.argv[2])
a, b = marks[-nst-1], marks[-1]
sel = rows[a+1:b+1]
t0 = int(rows[a]["End_Timestamp"]); t1 = int(rows[b]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"])-int(r["Start_Timestamp"]) for r in sel)
print(f"{nst} steps: {(t1-t0)/1e3/nst:.1f} us/step wall, {busy/1e3/nst:.1f} us busy, {len(sel)/nst:.1f} launches/step")
# one step list with gaps
one = rows[marks[-2]+1:marks[-1]+1]
prev = int(rows[marks[-2]]["End_Timestamp"])
for r in one:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"gap {(s-prev)/1e3:7.1f}  dur {(e-s)/1e3:7.1f}  {r['Kernel_Name'][:90]}")
    prev = e
