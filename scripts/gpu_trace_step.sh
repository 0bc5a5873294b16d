#!/bin/bash
# Kernel trace of the flagship bench (20 timed steps after 20 warmup) and the launch sequence of
# its median step per hardware queue (scripts/step_kernels.py) -> gpurun_out/ts/. Extra bench args
# in BENCH_ARGS. rocprofv3 may crash at teardown after writing its output: its status is not checked.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
O=${TS_OUT:-gpurun_out/ts}; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 20 ${BENCH_ARGS:-} > $O/trace.log 2>&1
python scripts/step_kernels.py $O/trace/run_kernel_trace.csv 19 > $O/step_kernels.txt 2>&1
head -6 $O/step_kernels.txt
exit 0
