#!/bin/bash
# Round 6, batch EV5: 16-bit record counts (params.h: 32-bit offsets, proteomes up to 32767 proteins),
# the chain's token layout capped at genome_pipeline.P_CAP proteins -- the whole GPU suite, the
# evolved-shape probe past the old 8191-protein limit, then evolved (3000 warmup) and fresh flagship
# runs of the tree against the previous commit (ab/head), interleaved.
set -o pipefail
O=$PWD/gpurun_out/r6ev5
mkdir -p $O
R=$PWD
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/lab/evo_shape.py 3000 > $O/shape.log 2>&1 || exit $?
for i in 1 2; do
  (cd $R && timeout -k 10 300 python -u bench.py --steps 100 --warmup 3000 > $O/ev_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 300 python -u bench.py --steps 100 --warmup 3000 > $O/ev_old_$i.log 2>&1) || exit $?
  (cd $R && timeout -k 10 300 python -u bench.py > $O/fresh_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 300 python -u bench.py > $O/fresh_old_$i.log 2>&1) || exit $?
done
