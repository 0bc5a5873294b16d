#!/bin/bash
# Default bench (20 + 60 steps): defaults vs initial arena headroom 2 + proactive widening,
# alternating, per-step times; then the slow-step events of the latter over 100 steps from the start.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/sab2; rm -rf $O; mkdir -p $O
for r in 1 2 3; do
  for v in "def:MS_GENOME_HEADROOM_INIT=1 MS_GENOME_WIDTH_WATCH=0" "hw:MS_GENOME_HEADROOM_INIT=2 MS_GENOME_WIDTH_WATCH=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 200 python bench.py --step-times > $O/${name}_r$r.log 2>&1
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
MS_GENOME_HEADROOM_INIT=2 MS_GENOME_WIDTH_WATCH=1 timeout -k 10 200 python scripts/spike_events.py 4096 50000 100 0 > $O/spikes_hw.log 2>&1
grep -c "restore" $O/spikes_hw.log
exit 0
