"""Gaps after k_mark_a in an event_lab.bin kernel trace: to k_next_wait (behind a cross-stream wait
on an already complete event) and to k_next_plain (no wait). Medians in microseconds.

    python scripts/lab/event_lab_report.py run_kernel_trace.csv
"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gaps = {"wait": [], "plain": []}
for i, r in enumerate(rows):
    if "k_mark_a" in r["Kernel_Name"]:
        end = int(r["End_Timestamp"])
        for q in rows[i + 1:]:
            if "k_next_wait" in q["Kernel_Name"]:
                gaps["wait"].append((int(q["Start_Timestamp"]) - end) / 1e3)
                break
            if "k_next_plain" in q["Kernel_Name"]:
                gaps["plain"].append((int(q["Start_Timestamp"]) - end) / 1e3)
                break
print({k: (round(statistics.median(v), 2), len(v)) for k, v in gaps.items() if v})
