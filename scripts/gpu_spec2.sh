#!/bin/bash
# Speculative integrator, LDS overflow route: kernel tests, a 300-step flagship run with per-step
# times and internal events (long-run genomes grow past the 64-lane slots), then the flagship bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/spec2; rm -rf $O; mkdir -p $O
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 "$O/$name.log" | cut -c1-300
  if fatal $rc; then echo "fatal rc=$rc in $name"; exit $rc; fi
  return $rc
}
run kernels 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "integrator or speculative or flags" || exit 1
run spikes 400 python scripts/spike_events.py 4096 50000 300 20
run bench_a 300 python bench.py
run bench_drv 300 python bench.py --steps 20 --warmup 5
exit 0
