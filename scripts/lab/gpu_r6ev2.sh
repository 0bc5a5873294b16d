#!/bin/bash
# Round 6, batch EV2: evolved flagship population (3000 warmup steps, 100 timed) -- the tree against
# the previous commit (ab/head: a worktree built in-tree) for the rescue launch's slot packing and the
# tighter protein bound, interleaved; then a kernel trace of 30 evolved steps of the tree.
set -o pipefail
O=$PWD/gpurun_out/r6ev2
mkdir -p $O
R=$PWD
for i in 1 2; do
  (cd $R && timeout -k 10 400 python -u bench.py --steps 100 --warmup 3000 > $O/ev_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 400 python -u bench.py --steps 100 --warmup 3000 > $O/ev_old_$i.log 2>&1) || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3000 > $O/kt.log 2>&1
