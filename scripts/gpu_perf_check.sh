#!/bin/bash
# Quick GPU perf loop: GPU tests, per-step times, a kernel trace and three clean bench runs.
# usage: scripts/gpu_perf_check.sh [tag]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag="${1:-pc}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --step-times > gpurun_out/${tag}_st.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --steps 10 --warmup 10 > gpurun_out/${tag}_rocprof.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 300 python bench.py --steps 60 --warmup 20 2>&1 | tail -1 | cut -c80-140 || exit 1; done
