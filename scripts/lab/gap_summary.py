"""Device idle gaps of a rocprofv3 kernel trace: which kernel launches the GPU waited for.

usage: python scripts/lab/gap_summary.py <kernel_trace.csv> [last_n_kernels]
Each gap between the end of one kernel and the start of the next is attributed to the pair
(previous -> next); host-side syncs and Python time between launches show up as large gaps."""
import collections
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:48])
              for r in csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
rows = rows[-n:]
gaps = collections.defaultdict(list)
end = rows[0][1]
for (s, e, k), (ps, pe, pk) in zip(rows[1:], rows[:-1]):
    g = s - max(pe, end)
    end = max(end, e)
    if g > 0:
        gaps[(pk, k)].append(g)
tot = sum(sum(v) for v in gaps.values())
span = rows[-1][1] - rows[0][0]
print(f"span {span / 1e6:.2f} ms, idle {tot / 1e6:.2f} ms over {len(rows)} kernels")
for (pk, k), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:30]:
    print(f"{sum(v) / 1e3:9.1f} us {len(v):5d}x  {pk} -> {k}")
