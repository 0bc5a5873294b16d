#!/bin/bash
# Round 6, batch Y: the flagship as one virtual strip with the early stencil (stencil before the wait,
# phase B on the side stream) allowed at 4096^2 (MS_EARLY_STENCIL_MAX_PX) against the default.
set -o pipefail
O=gpurun_out/r6y
mkdir -p $O
for i in 1 2 3; do
  MS_VIRTUAL_STRIPS=1 MS_EARLY_STENCIL_MAX_PX=100000000 timeout -k 10 200 python -u bench.py > $O/fv_early_$i.log 2>&1 || exit $?
  MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py > $O/fv_default_$i.log 2>&1 || exit $?
done
timeout -k 10 200 python -u bench.py > $O/flag.log 2>&1
