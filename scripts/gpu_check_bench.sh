#!/bin/bash
# Quick GPU check: selected GPU tests (pytest -k expression in $1, optional) and N flagship bench
# runs (default 3) as the driver runs them (no per-step synchronisation); each step under its own
# time limit, stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
O=gpurun_out/chk
mkdir -p $O
if [ -n "${1:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for i in $(seq 1 ${2:-3}); do
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/b$i.log 2>&1 || exit 1
  python - $O/b$i.log <<'PY'
import json, statistics, sys
for l in open(sys.argv[1]):
    if l.startswith('{"step_ms'):
        v = json.loads(l)["step_ms"]
        print(f"  steps: median {statistics.median(v):.3f} ms, min {min(v):.3f}, max {max(v):.3f}")
    if l.startswith('{"metric'):
        d = json.loads(l)
        print(f"  {d['value']} steps/s, {d['ms_per_step']} ms/step, cells {d['config']['cells_at_end']}")
PY
done
