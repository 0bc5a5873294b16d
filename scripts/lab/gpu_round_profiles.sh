#!/bin/bash
# End-of-round evidence: BASELINE configs, the reference macro config, PMC counter groups and a
# host profile; each GPU step under its own time limit, stop at the first fatal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
bash scripts/lab/gpu_configs.sh configs || exit $?
timeout -k 10 300 python bench.py --map-size 256 --cells 40000 --steps 60 --warmup 20 > gpurun_out/configs/c256_40k.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 60 --warmup 20 > gpurun_out/configs/c4096_50k.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 60 --warmup 20 --map-dtype bf16 > gpurun_out/configs/c4096_50k_bf16.log 2>&1 || exit $?
bash scripts/lab/gpu_counters.sh > gpurun_out/pmc_run.log 2>&1 || exit $?
timeout -k 10 300 python scripts/lab/profile_step.py 4096 50000 20 > gpurun_out/cprofile_4096_50k.log 2>&1
