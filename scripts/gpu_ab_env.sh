#!/bin/bash
# A/B of an environment setting on the flagship bench: alternating runs with and without "$1"
# (e.g. HIP_FORCE_DEV_KERNARG=0), $2 pairs (default 3); extra bench args in BENCH_ARGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
O=gpurun_out/ab; mkdir -p $O
for i in $(seq 1 ${2:-3}); do
  for v in base alt; do
    if [ $v = alt ]; then E="env $1"; else E=""; fi
    timeout -k 10 300 $E python bench.py --step-times ${BENCH_ARGS:-} > $O/$v$i.log 2>&1 || exit 1
    python - $O/$v$i.log $v <<'PY'
import json, statistics, sys
med = val = None
for l in open(sys.argv[1]):
    if l.startswith('{"step_ms'):
        med = statistics.median(json.loads(l)["step_ms"])
    if l.startswith('{"metric'):
        val = json.loads(l)["value"]
print(f"  {sys.argv[2]:4s} {val} steps/s, median step {med:.3f} ms")
PY
  done
done
