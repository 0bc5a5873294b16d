#!/bin/bash
# Initial genome-arena headroom (MS_GENOME_HEADROOM_INIT) A/B on the driver-style run (5 + 20 steps)
# and the default bench, alternating processes, per-step times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/hr0; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for h in 1 2; do
    for cfg in "20 5" "60 20"; do
      st=${cfg% *}; wu=${cfg#* }
      MS_GENOME_HEADROOM_INIT=$h timeout -k 10 200 python bench.py --steps $st --warmup $wu --step-times > $O/h${h}_s${st}_r$r.log 2>&1
      rc=$?
      python - "$O/h${h}_s${st}_r$r.log" <<'PY'
import json, statistics, sys
t = open(sys.argv[1]).read()
st = json.loads(t[t.index('{"step_ms"'):].splitlines()[0])["step_ms"]
v = json.loads(t[t.index('{"metric"'):].splitlines()[0])["value"]
print(sys.argv[1].split("/")[-1], "value", v, "median", statistics.median(st), "max", max(st), "first4", st[:4])
PY
      case $rc in 124|134|137|139) exit $rc;; esac
    done
  done
done
exit 0
