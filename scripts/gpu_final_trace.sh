#!/bin/bash
# Kernel trace + stats of the flagship bench on the current tree (20 warmup + 20 timed steps) and
# the median step's launch sequence per queue. rocprofv3 may crash at teardown after writing its
# output: its exit status is not checked.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/ft; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 20 > $O/trace.log 2>&1
python scripts/step_kernels.py $O/trace/run_kernel_trace.csv 19 > $O/step_kernels.txt 2>&1
head -6 $O/step_kernels.txt
exit 0
