#!/bin/bash
# Genome-arena headroom (MS_GENOME_HEADROOM) x eager genome chains (MS_EAGER_CHAINS): per-step times
# of the default bench and of the driver-style run for each setting.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/hr; rm -rf $O; mkdir -p $O
for v in "1 0" "2 0" "4 0" "1 1"; do
  set -- $v
  for cfg in "60 20" "20 5"; do
    st=${cfg% *}; wu=${cfg#* }
    MS_GENOME_HEADROOM=$1 MS_EAGER_CHAINS=$2 timeout -k 10 200 python bench.py --steps $st --warmup $wu --step-times > $O/hr$1_e$2_s$st.log 2>&1
    rc=$?
    python - "$O/hr$1_e$2_s$st.log" <<'PY'
import json, statistics, sys
t = open(sys.argv[1]).read()
st = json.loads(t[t.index('{"step_ms"'):].splitlines()[0])["step_ms"]
v = json.loads(t[t.index('{"metric"'):].splitlines()[0])["value"]
print(sys.argv[1].split("/")[-1], "value", v, "median", statistics.median(st), "mean", round(sum(st) / len(st), 3))
PY
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
