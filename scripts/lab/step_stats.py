"""Summarise a bench --step-times log: median / mean / spikes."""
import json
import re
import statistics
import sys

v = json.loads(re.search(r'\{"step_ms": \[[^\]]*\]\}', open(sys.argv[1]).read()).group(0))["step_ms"]
print(f"n={len(v)} median={statistics.median(v):.3f} mean={statistics.mean(v):.3f} max={max(v):.3f}")
print(" ".join(f"{x:.2f}" for x in v))
