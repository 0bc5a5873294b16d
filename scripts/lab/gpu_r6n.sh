#!/bin/bash
# Round 6, batch N: host split of the virtual-strip and plain N = 8 proxies with graph batching on and
# off (per native entry point), with the per-step batch statistics.
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
for g in 1 0; do
  MS_GRAPH_BATCH=$g MS_VIRTUAL_STRIPS=1 MS_NATIVE_TIMES=1 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hsv_g$g.log 2>&1 || exit $?
  MS_GRAPH_BATCH=$g MS_NATIVE_TIMES=1 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hsp_g$g.log 2>&1 || exit $?
  MS_GRAPH_BATCH=$g MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hsv_plain_timing_g$g.log 2>&1 || exit $?
done
