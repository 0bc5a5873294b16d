#!/bin/bash
# Final check of a tree: GPU suite + smoke, then driver-style and default flagship benches (three
# and two runs) with per-step times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/final; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for r in 1 2 3; do
  for cfg in "20 5" "60 20"; do
    st=${cfg% *}; wu=${cfg#* }
    [ "$r" = 3 ] && [ "$st" = 60 ] && continue
    timeout -k 10 200 python bench.py --steps $st --warmup $wu --step-times > $O/s${st}_r$r.log 2>&1
    rc=$?
    python - "$O/s${st}_r$r.log" <<'PY'
import json, statistics, sys
t = open(sys.argv[1]).read()
st = json.loads(t[t.index('{"step_ms"'):].splitlines()[0])["step_ms"]
v = json.loads(t[t.index('{"metric"'):].splitlines()[0])["value"]
print(sys.argv[1].split("/")[-1], "value", v, "median", statistics.median(st), "max", max(st), "first4", st[:4])
PY
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
exit 0
