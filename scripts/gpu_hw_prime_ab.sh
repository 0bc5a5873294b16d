#!/bin/bash
# With priming in place: driver-style runs with the short-warm-up reservation (hw, bench default)
# vs without it (MS_GENOME_HEADROOM_INIT=1 MS_GENOME_WIDTH_WATCH=0), five alternating pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/hwp; rm -rf $O; mkdir -p $O
for r in 1 2 3 4 5; do
  for v in "hw:MS_NOOP=1" "plain:MS_GENOME_HEADROOM_INIT=1 MS_GENOME_WIDTH_WATCH=0"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --step-times > $O/${name}_r$r.log 2>&1
    rc=$?
    python - "$O/${name}_r$r.log" <<'PY'
import json, statistics, sys
t = open(sys.argv[1]).read()
st = json.loads(t[t.index('{"step_ms"'):].splitlines()[0])["step_ms"]
v = json.loads(t[t.index('{"metric"'):].splitlines()[0])["value"]
print(sys.argv[1].split("/")[-1], "value", v, "median", statistics.median(st), "max", max(st))
PY
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
