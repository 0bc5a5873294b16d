#!/bin/bash
# GPU-box check: tests, smoke, benches. Each GPU step has its own time limit; a crash, abort or
# timeout (exit 124/134/137/139) ends the script without starting further GPU work.
# usage: scripts/lab/gpu_check.sh [tests|bench|all] [extra bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
what="${1:-all}"; shift || true
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name" | tee -a gpurun_out/summary.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$name.log" | tee -a gpurun_out/summary.log
  if fatal $rc; then echo "fatal rc=$rc in $name, stopping" | tee -a gpurun_out/summary.log; exit $rc; fi
  return 0
}
python -c "import __graft_entry__ as g; g.build()" || exit 1
if [[ "$what" == tests || "$what" == all ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ "$what" == bench || "$what" == all ]]; then
  # clean runs (the driver's measurement), then a phase breakdown (timers + event counts add syncs)
  run bench_256_40k 600 python bench.py --map-size 256 --cells 40000 --steps 30 --warmup 5 "$@"
  run bench_4096_50k 600 python bench.py --steps 30 --warmup 5 "$@"
  run bench_4096_50k_phases 600 python bench.py --steps 20 --warmup 5 --profile-phases "$@"
fi
if [[ "$what" == lowp ]]; then
  run pytest_maps 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q -k "diffusion or reduced or bf16 or permeation"
  run bench_4096_50k 600 python bench.py --steps 30 --warmup 5 "$@"
  run bench_4096_50k_bf16 600 python bench.py --steps 30 --warmup 5 --map-dtype bf16 "$@"
  run bench_4096_50k_phases 600 python bench.py --steps 20 --warmup 5 --profile-phases "$@"
fi
