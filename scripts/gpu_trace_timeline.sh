#!/bin/bash
# HIP API + kernel trace of the flagship bench and the host / device timeline of its fastest and
# slowest timed step (scripts/host_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/tl
rm -rf $O; mkdir -p $O
# rocprofv3 may crash at teardown after writing its output: its exit status is not checked
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 20 ${BENCH_ARGS:-} > $O/trace.log 2>&1
python scripts/host_timeline.py $O/trace 20 fast > $O/timeline_fast.txt 2>&1
python scripts/host_timeline.py $O/trace 20 slow > $O/timeline_slow.txt 2>&1
head -2 $O/timeline_fast.txt
exit 0
