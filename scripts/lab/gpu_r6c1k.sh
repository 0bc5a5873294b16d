#!/bin/bash
# Round 6, C1K: the small host-bound c1024 preset, the tree against the commit before the genome
# pipeline's scratch bound (ab/head), interleaved -- does the bound's host work show?
set -o pipefail
O=$PWD/gpurun_out/r6c1k
mkdir -p $O
R=$PWD
for i in 1 2 3; do
  (cd $R && timeout -k 10 200 python -u bench.py --preset c1024 --steps 30 --warmup 5 > $O/new_$i.log 2>&1) || exit $?
  (cd $R/ab/head && timeout -k 10 200 python -u bench.py --preset c1024 --steps 30 --warmup 5 > $O/old_$i.log 2>&1) || exit $?
done
