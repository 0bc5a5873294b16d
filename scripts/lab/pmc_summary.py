"""Per-kernel averages of a rocprofv3 --pmc counter collection (one CSV per counter pass).

usage: python scripts/lab/pmc_summary.py gpurun_out/pmc/g*/run_counter_collection.csv"""
import collections
import csv
import sys


def main():
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.defaultdict(int))
    dur = collections.defaultdict(list)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
            c = r["Counter_Name"]
            tot[k][c] += float(r["Counter_Value"])
            cnt[k][c] += 1
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k in sorted(tot):
        d = {c: tot[k][c] / cnt[k][c] for c in tot[k]}
        us = sum(dur[k]) / len(dur[k]) / 1e3
        print(f"== {k}  (mean dispatch {us:.1f} us under counters)")
        for c in sorted(d):
            print(f"   {c:28s} {d[c]:16.1f}")
        if "SQ_ACTIVE_INST_VALU" in d and "SQ_BUSY_CYCLES" in d:
            pass
        if "FETCH_SIZE" in d:
            print(f"   -> fetched {d['FETCH_SIZE'] / 1024:.1f} MiB per dispatch")
        if "WRITE_SIZE" in d:
            print(f"   -> wrote   {d['WRITE_SIZE'] / 1024:.1f} MiB per dispatch")
        if "SQ_WAIT_INST_ANY" in d and "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            print(f"   -> waiting on instructions/memory {100 * d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES']:.0f}% of wave cycles")


if __name__ == "__main__":
    main()
