#!/bin/bash
# Early diffusion stencil: its tests and the full GPU suite, then the flagship bench with and without
# it (MS_EARLY_DIFFUSE=0) and a kernel trace of the median step. Every GPU step has its own time
# limit; a fatal exit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/early; rm -rf $O; mkdir -p $O
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
run early_tests 300 python -u -m pytest tests/test_gpu_early_diffusion.py -x -v --timeout 120 --timeout-method thread || exit 1
run gpu_suite 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
run bench_early_a 300 python bench.py
MS_EARLY_DIFFUSE=0 run bench_late_a 300 python bench.py
run bench_early_b 300 python bench.py
MS_EARLY_DIFFUSE=0 run bench_late_b 300 python bench.py
run bench_drv 300 python bench.py --steps 20 --warmup 5
run bench_256 300 python bench.py --map-size 256 --cells 40000
TS_OUT=$O/ts bash scripts/gpu_trace_step.sh > $O/trace_step.log 2>&1
exit 0
