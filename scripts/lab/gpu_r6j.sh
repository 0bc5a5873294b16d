#!/bin/bash
# Round 6, batch J: the round-5 tree (ab/r5, a git worktree of 8264e4a built in-tree) against the
# current tree on the same box: the N = 8 per-rank proxy plain and as a virtual strip, interleaved,
# plus kernel traces of both virtual runs.
set -o pipefail
O=$PWD/gpurun_out/r6j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
R=$PWD
for i in 1 2; do
  for t in cur r5; do
    d=$R; [ $t = r5 ] && d=$R/ab/r5
    (cd $d && timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/plain_${t}_$i.log 2>&1) || exit $?
    (cd $d && MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/virt_${t}_$i.log 2>&1) || exit $?
  done
done
for t in cur r5; do
  d=$R; [ $t = r5 ] && d=$R/ab/r5
  (cd $d && MS_VIRTUAL_STRIPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_virt_$t -o run --output-format csv -- python3 bench.py --map-size 1448 --cells 6250 > $O/kt_virt_$t.log 2>&1) || exit $?
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_plain_$t -o run --output-format csv -- python3 bench.py --map-size 1448 --cells 6250 > $O/kt_plain_$t.log 2>&1) || exit $?
done
