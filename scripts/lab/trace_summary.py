"""Summarise a rocprofv3 kernel trace over the timed steps of a bench run.

usage: python scripts/lab/trace_summary.py <kernel_trace.csv> <n_timed_steps>
           [--marker-csv run_marker_api_trace.csv] [--marker integrate_part_kernel --per-step 3]

Kernels after the last (n_timed_steps * per_step) launches of the marker kernel's step are
attributed to the timed steps. With a roctx marker trace of a ``--profile-phases --phase-sync``
bench run (MS_ROCTX=1), kernels are also attributed to the phase ranges that contain them."""
import argparse
import collections
import csv


def _ranges(path):
    out = []
    for r in csv.DictReader(open(path)):
        name = r.get("Function") or r.get("Marker_Name") or r.get("Name") or ""
        try:
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
        except (KeyError, ValueError):
            continue
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("steps", type=int)
    ap.add_argument("--marker-csv")
    ap.add_argument("--marker", default="integrate_part_kernel")
    ap.add_argument("--per-step", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(a.marker)]
    n = a.steps * a.per_step
    start = marks[-n - 1] + 1 if len(marks) > n else 0
    sel = rows[start:]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"].split("(")[0][:70]
        agg[name][0] += 1
        agg[name][1] += d
        busy += d
    st = a.steps
    print(f"window {(t1 - t0) / 1e6:.2f} ms over {st} steps: {(t1 - t0) / 1e6 / st:.3f} ms/step wall, "
          f"{busy / 1e3 / st:.3f} ms/step kernel busy, {len(sel) / st:.0f} launches/step")
    print(f"{'us/step':>9} {'calls/step':>10} {'us/call':>8}  kernel")
    for name, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{d / st:9.1f} {c / st:10.1f} {d / c:8.1f}  {name}")
    if not a.marker_csv:
        return
    ranges = [rg for rg in _ranges(a.marker_csv) if rg[1] >= t0 and rg[0] <= t1]
    phases = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
    for r in sel:
        ks, ke = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        best = None
        for rs, re_, nm in ranges:  # innermost containing range
            if rs <= ks and ke <= re_ and (best is None or re_ - rs < best[1] - best[0]):
                best = (rs, re_, nm)
        ph = best[2] if best else "(none)"
        e = phases[ph][r["Kernel_Name"].split("(")[0][:60]]
        e[0] += 1
        e[1] += (ke - ks) / 1e3
    print("\nper phase (innermost roctx range):")
    for ph, ks in sorted(phases.items(), key=lambda kv: -sum(v[1] for v in kv[1].values())):
        tot = sum(v[1] for v in ks.values())
        cnt = sum(v[0] for v in ks.values())
        print(f"== {ph}: {tot / st:.1f} us/step kernel busy, {cnt / st:.1f} launches/step")
        for name, (c, d) in sorted(ks.items(), key=lambda kv: -kv[1][1])[:8]:
            print(f"   {d / st:8.1f} us {c / st:6.1f}x  {name}")


if __name__ == "__main__":
    main()
