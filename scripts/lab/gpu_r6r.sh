#!/bin/bash
# Round 6, batch R: the strip stencil issued before the wait for phase A's counts. Strip GPU tests,
# then the N = 8 virtual proxy and the flagship as one strip with the knob on / off, interleaved.
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_kernels.py -k "strip or distributed or lazy or rccl" -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit $?
for i in 1 2 3; do
  for k in 1 0; do
    MS_STENCIL_BEFORE_WAIT=$k MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/virt8_k${k}_$i.log 2>&1 || exit $?
  done
done
for i in 1 2; do
  for k in 1 0; do
    MS_STENCIL_BEFORE_WAIT=$k MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py > $O/flagvirt_k${k}_$i.log 2>&1 || exit $?
  done
done
