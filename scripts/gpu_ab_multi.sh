#!/bin/bash
# A/B/C... of environment settings on the flagship bench: for each of $2 rounds, one run per
# setting in $1 (space-separated; "base" = no setting), alternating; extra bench args in BENCH_ARGS.
# e.g. bash scripts/gpu_ab_multi.sh "base MS_STENCIL_BLOCKS=0 MS_STENCIL_BLOCKS=1024" 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
O=gpurun_out/abm; mkdir -p $O
for i in $(seq 1 ${2:-3}); do
  for v in $1; do
    if [ $v = base ]; then E=""; else E="env $v"; fi
    timeout -k 10 300 $E python bench.py --step-times ${BENCH_ARGS:-} > $O/$v.$i.log 2>&1 || exit 1
    python - $O/$v.$i.log $v <<'PY'
import json, statistics, sys
med = val = None
for l in open(sys.argv[1]):
    if l.startswith('{"step_ms'):
        med = statistics.median(json.loads(l)["step_ms"])
    if l.startswith('{"metric'):
        val = json.loads(l)["value"]
print(f"  {sys.argv[2]:28s} {val} steps/s, median step {med:.3f} ms")
PY
  done
done
