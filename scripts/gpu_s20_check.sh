#!/bin/bash
# Driver-style runs (5 + 20 steps) x6 and default runs x2 of the current tree, per-step times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/s20; rm -rf $O; mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  args="--steps 20 --warmup 5"; [ $r -gt 6 ] && args=""
  timeout -k 10 200 python bench.py $args --step-times > $O/r$r.log 2>&1
  rc=$?
  python - "$O/r$r.log" "$args" <<'PY'
import json, statistics, sys
t = open(sys.argv[1]).read()
st = json.loads(t[t.index('{"step_ms"'):].splitlines()[0])["step_ms"]
v = json.loads(t[t.index('{"metric"'):].splitlines()[0])["value"]
print(sys.argv[1].split("/")[-1], sys.argv[2] or "default", "value", v, "median", statistics.median(st), "max", max(st))
PY
  case $rc in 124|134|137|139) exit $rc;; esac
done
exit 0
