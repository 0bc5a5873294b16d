#!/bin/bash
# Round 6, batch EV8: long-genome translation pass sorting CDS lists in LDS (genetics.hip kSortCap; a
# first try batching phase-1/2 loads was 5 % slower and dropped) -- translation / pipeline GPU tests, the long-genome translation
# micro-bench (tree and ab/head), then evolved (3000 warmup) and fresh flagship runs vs ab/head.
set -o pipefail
O=$PWD/gpurun_out/r6ev8
mkdir -p $O
R=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "genome_pipeline or merged or speculative or translation or param_build or huge or bench_steps" > $O/tests.log 2>&1 || exit $?
(cd $R && timeout -k 10 300 python -u scripts/lab/tlong_bench.py > $O/tl_new.log 2>&1) || exit $?
(cd $R/ab/head && timeout -k 10 300 python -u $R/scripts/lab/tlong_bench.py > $O/tl_old.log 2>&1) || exit $?
for i in 1 2; do
  (cd $R && timeout -k 10 300 python -u bench.py --steps 100 --warmup 3000 > $O/ev_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 300 python -u bench.py --steps 100 --warmup 3000 > $O/ev_old_$i.log 2>&1) || exit $?
  (cd $R && timeout -k 10 300 python -u bench.py > $O/fresh_new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 300 python -u bench.py > $O/fresh_old_$i.log 2>&1) || exit $?
done
