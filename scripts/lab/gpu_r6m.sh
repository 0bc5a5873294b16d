#!/bin/bash
# Round 6, batch M: graph-batched launches (csrc/hip/launch.h). GPU suite, then the flagship and the
# N = 8 per-rank proxies with batching on and off (MS_GRAPH_BATCH=0), interleaved.
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
for i in 1 2; do
  for g in 1 0; do
    MS_GRAPH_BATCH=$g timeout -k 10 200 python -u bench.py > $O/flag_g${g}_$i.log 2>&1 || exit $?
    MS_GRAPH_BATCH=$g timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/plain8_g${g}_$i.log 2>&1 || exit $?
    MS_GRAPH_BATCH=$g MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/virt8_g${g}_$i.log 2>&1 || exit $?
  done
done
