"""Host / device timeline of one bench step from a rocprofv3 ``--hip-trace --kernel-trace`` CSV pair:
every HIP API call that launches, copies or waits (host time relative to the step start, its
duration) next to the kernel it launched (device start relative to the step start, duration), and
per-step totals: host time blocked in synchronisations and device idle time.

usage: python scripts/host_timeline.py <dir with run_hip_api_trace.csv / run_kernel_trace.csv> [steps] [which]
    which: last (default) | fast | slow -- the step whose call list is printed"""
import csv
import os
import sys

d = sys.argv[1]
nst = int(sys.argv[2]) if len(sys.argv) > 2 else 10
api = [r for r in csv.DictReader(open(os.path.join(d, "run_hip_api_trace.csv")))]
ker = sorted(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
by_corr = {r["Correlation_Id"]: r for r in ker}
NOISE = {"hipGetDevice", "hipSetDevice", "hipGetLastError", "__hipPushCallConfiguration",
         "__hipPopCallConfiguration", "hipStreamIsCapturing", "hipStreamGetCaptureInfo",
         "hipDevicePrimaryCtxGetState", "__hipRegisterFunction", "__hipRegisterFatBinary", "__hipRegisterVar"}
SYNC = {"hipStreamSynchronize", "hipEventSynchronize", "hipDeviceSynchronize", "hipMemcpyWithStream", "hipMemcpy"}
api = sorted((r for r in api if r["Function"] not in NOISE), key=lambda r: int(r["Start_Timestamp"]))
marks = [r for r in api if r["Correlation_Id"] in by_corr
         and by_corr[r["Correlation_Id"]]["Kernel_Name"].startswith("void msd::diffuse_stencil4")]
steps = []
for a, b in zip(marks[-nst - 1:-1], marks[-nst:]):
    t0, t1 = int(a["End_Timestamp"]), int(b["End_Timestamp"])
    steps.append((t0, t1, [r for r in api if t0 < int(r["Start_Timestamp"]) <= t1]))
tot_sync = tot_wall = tot_idle = 0
for t0, t1, calls in steps:
    sync = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in calls if r["Function"] in SYNC)
    ks = sorted((by_corr[r["Correlation_Id"]] for r in calls if r["Correlation_Id"] in by_corr),
                key=lambda k: int(k["Start_Timestamp"]))
    busy = sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks)
    tot_sync += sync
    tot_wall += t1 - t0
    tot_idle += (t1 - t0) - busy
print(f"{nst} steps: host wall {tot_wall / nst / 1e3:.1f} us/step, blocked in syncs {tot_sync / nst / 1e3:.1f} us, "
      f"device idle (approx) {tot_idle / nst / 1e3:.1f} us")
which = sys.argv[3] if len(sys.argv) > 3 else "last"
if which == "fast":
    t0, t1, calls = min(steps, key=lambda st: st[1] - st[0])
elif which == "slow":
    t0, t1, calls = max(steps, key=lambda st: st[1] - st[0])
else:
    t0, t1, calls = steps[-1]
print(f"step walls (us): {' '.join(str((b - a) // 1000) for a, b, _ in steps)}; showing {which}: {(t1 - t0) / 1e3:.1f} us")
print(f"{'host_t':>8s} {'dur':>7s}  {'call':24s} {'dev_t':>8s} {'kdur':>7s}  kernel")
for r in calls:
    hs, he = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    k = by_corr.get(r["Correlation_Id"])
    ks = kd = ""
    name = ""
    if k is not None:
        ks = f"{(int(k['Start_Timestamp']) - t0) / 1e3:8.1f}"
        kd = f"{(int(k['End_Timestamp']) - int(k['Start_Timestamp'])) / 1e3:7.1f}"
        name = k["Kernel_Name"][:70]
    print(f"{hs / 1e3:8.1f} {he / 1e3:7.1f}  {r['Function'][:24]:24s} {ks:>8s} {kd:>7s}  {name}")
