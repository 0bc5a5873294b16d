"""HIP API calls and kernels per step from a rocprofv3 ``--hip-trace --kernel-trace`` run of bench.py.

Steps are delimited by the permeation kernel (one launch per step, plain and strip worlds alike);
the last 40 steps are summarised: HIP API calls of the main thread per step (count, host µs under
the tracer -- the tracer inflates every call) and kernels per step by name.

usage: python scripts/lab/hip_api_per_step.py <rocprofv3 output dir holding run_hip_api_trace.csv and
run_kernel_trace.csv> [steps]"""
import collections
import csv
import sys

d = sys.argv[1]
nst = int(sys.argv[2]) if len(sys.argv) > 2 else 40
api = list(csv.DictReader(open(d + "/run_hip_api_trace.csv")))
kt = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
marks = sorted(int(r["Correlation_Id"]) for r in kt if "permeate_kernel" in r["Kernel_Name"])
kn = {int(r["Correlation_Id"]): r["Kernel_Name"] for r in kt}
lo, hi = marks[-nst - 1], marks[-1]
calls, host = collections.Counter(), collections.Counter()
for r in api:
    cid = int(r["Correlation_Id"])
    if lo <= cid < hi and r["Thread_Id"] == r["Process_Id"]:
        f = r["Function"]
        calls[f] += 1
        host[f] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
ks = collections.Counter(kn[k].split("(")[0][:60] for k in kn if lo <= k < hi)
print("per step (main thread), calls / host us:")
for f, n in calls.most_common(25):
    print(f"  {f:40s} {n / nst:6.1f} {host[f] / nst / 1000:8.1f}")
print("kernels per step:", sum(ks.values()) / nst)
for k, n in ks.most_common(60):
    print(f"  {n / nst:5.2f} {k}")
