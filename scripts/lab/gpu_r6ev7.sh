#!/bin/bash
# Round 6, batch EV7: recombination / mutation byte copies with eight loads in flight per lane
# (rec_common.h wave_copy) -- the whole GPU suite, then evolved (3000 warmup) and fresh flagship runs
# of the tree against ab/head (the previous commit), interleaved, and a kernel trace of 30 evolved steps.
set -o pipefail
O=$PWD/gpurun_out/r6ev7
mkdir -p $O
R=$PWD
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || exit $?
for i in 1 2; do
  (cd $R && timeout -k 10 300 python -u bench.py --steps 100 --warmup 3000 > $O/ev_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 300 python -u bench.py --steps 100 --warmup 3000 > $O/ev_old_$i.log 2>&1) || exit $?
  (cd $R && timeout -k 10 300 python -u bench.py > $O/fresh_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 300 python -u bench.py > $O/fresh_old_$i.log 2>&1) || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 30 --warmup 3000 > $O/kt.log 2>&1
