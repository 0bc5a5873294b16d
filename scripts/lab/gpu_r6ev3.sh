#!/bin/bash
# Round 6, batch EV3: per-cell overflow list of the rebuild chain (gp.hip gp_check_assign_kernel) --
# the genome-pipeline GPU tests, then the evolved flagship population (3000 warmup steps, 100 timed)
# of the tree against the previous commit (ab/head: a worktree built in-tree), interleaved; then a
# kernel trace of 30 evolved steps of the tree.
set -o pipefail
O=$PWD/gpurun_out/r6ev3
mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "genome_pipeline or merged or speculative or translation or param_build or huge" > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  (cd $R && timeout -k 10 400 python -u bench.py --steps 100 --warmup 3000 > $O/ev_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 400 python -u bench.py --steps 100 --warmup 3000 > $O/ev_old_$i.log 2>&1) || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3000 > $O/kt.log 2>&1
