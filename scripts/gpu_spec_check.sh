#!/bin/bash
# Speculative all-parts integrator: kernel tests, then the integrator A/B on the flagship state and
# the flagship bench with and without the speculative launch (MS_INTEGRATE_MODE=128). Every GPU step
# has its own time limit; a fatal exit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
O=gpurun_out/spec; rm -rf $O; mkdir -p $O
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log"
  if fatal $rc; then echo "fatal rc=$rc in $name"; exit $rc; fi
  return $rc
}
run kernels 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "integrator or speculative or flags" || exit 1
run integrator_ab 300 python scripts/integrator_bench.py
run bench_spec_a 300 python bench.py
MS_INTEGRATE_MODE=128 run bench_perpart_a 300 python bench.py
run bench_spec_b 300 python bench.py
MS_INTEGRATE_MODE=128 run bench_perpart_b 300 python bench.py
run bench_drv 300 python bench.py --steps 20 --warmup 5
exit 0
