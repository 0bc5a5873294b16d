#!/bin/bash
# Host-side evidence for the per-step host floor: a HIP API + kernel trace of the flagship bench
# (scripts/host_timeline.py reads it), cProfiles of single World ops, and two plain bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tl
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/tl
timeout -k 10 300 python bench.py > $O/bench_a.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench_b.log 2>&1 || exit 1
grep -h '^{"metric"' $O/bench_a.log $O/bench_b.log | cut -c1-200
for op in mutate recombinate divide50; do
  timeout -k 10 200 python scripts/op_cprofile.py $op 200 > $O/cp_$op.txt 2>&1 || exit 1
done
timeout -k 10 200 python scripts/op_cprofile.py kill50 200 30000 > $O/cp_kill50.txt 2>&1 || exit 1
# rocprofv3 may crash at teardown after writing its output: its exit status is not checked
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/trace -o run --output-format csv -- python bench.py --steps 10 --warmup 20 > $O/trace.log 2>&1
python scripts/host_timeline.py $O/trace 10 > $O/timeline.txt 2>&1
head -3 $O/timeline.txt
exit 0
