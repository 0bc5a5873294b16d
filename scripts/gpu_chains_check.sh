#!/bin/bash
# Eager genome chains (lazy join) + genome-arena headroom: GPU suite, paired in-process A/B of the
# chain issue points, the driver-style bench (20 + 5 steps) three times and the default bench twice,
# one of them with the previous behaviour (MS_EAGER_CHAINS=0 MS_GENOME_HEADROOM=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/chains; rm -rf $O; mkdir -p $O
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc $(grep -ho '"value": [0-9.]*' $O/$name.log)"; tail -2 "$O/$name.log" | cut -c1-250
  if fatal $rc; then echo "fatal rc=$rc in $name"; exit $rc; fi
  return $rc
}
run gpu_suite 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread || exit 1
run ab 300 python scripts/early_ab.py 4096 50000 8 10
run drv1 200 python bench.py --steps 20 --warmup 5 --step-times
run drv2 200 python bench.py --steps 20 --warmup 5 --step-times
run drv3 200 python bench.py --steps 20 --warmup 5 --step-times
run def_new 200 python bench.py
MS_EAGER_CHAINS=0 MS_GENOME_HEADROOM=1 run def_old 200 python bench.py
run def_new2 200 python bench.py
MS_EAGER_CHAINS=0 MS_GENOME_HEADROOM=1 run drv_old 200 python bench.py --steps 20 --warmup 5 --step-times
exit 0
