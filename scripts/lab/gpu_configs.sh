#!/bin/bash
# The BASELINE.json configs on one MI355X, plus the reference's per-op and macro workloads.
# Each GPU step has its own time limit; a crash, abort or timeout ends the script.
# usage: scripts/lab/gpu_configs.sh [configs|perf|all]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/configs
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
what="${1:-all}"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name" | tee -a gpurun_out/configs/summary.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/configs/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/configs/summary.log
  tail -3 "gpurun_out/configs/$name.log" | tee -a gpurun_out/configs/summary.log
  if fatal $rc; then echo "fatal rc=$rc in $name, stopping" | tee -a gpurun_out/configs/summary.log; exit $rc; fi
  return 0
}
if [[ "$what" == configs || "$what" == all ]]; then
  run c1024_10k_16x32_bf16 400 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --map-dtype bf16 --steps 30 --warmup 5
  run c1024_10k_16x32_fp32 400 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --steps 30 --warmup 5
  run c4096_50k_64x256 400 python bench.py --map-size 4096 --cells 50000 --chemistry synthetic:64:256 --steps 20 --warmup 5
  run c16384_1m_fp16 600 python bench.py --map-size 16384 --cells 1000000 --map-dtype fp16 --steps 10 --warmup 3
fi
if [[ "$what" == perf || "$what" == all ]]; then
  run check_py 600 python performance/check.py --device cuda
  run run_simulation 600 python performance/run_simulation.py --device cuda --n-steps 200
fi
