#!/bin/bash
# Proactive genome-arena widening (MS_GENOME_WIDTH_WATCH): slow-step events over 100 steps from the
# start, then driver-style and default bench runs with and without it (alternating), per-step times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/ww; rm -rf $O; mkdir -p $O
timeout -k 10 200 python scripts/spike_events.py 4096 50000 100 0 > $O/spikes.log 2>&1 || exit $?
head -40 $O/spikes.log | cut -c1-200
for r in 1 2; do
  for h in 1 0; do
    for cfg in "20 5" "60 20"; do
      st=${cfg% *}; wu=${cfg#* }
      MS_GENOME_WIDTH_WATCH=$h timeout -k 10 200 python bench.py --steps $st --warmup $wu --step-times > $O/w${h}_s${st}_r$r.log 2>&1
      rc=$?
      python - "$O/w${h}_s${st}_r$r.log" <<'PY'
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
