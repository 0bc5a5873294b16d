#!/bin/bash
# Round 6, batch A: new GPU tests (torch oracles, totals, payload selection), the m1 config's N = 8
# per-rank share (5793^2 / 125k cells, fp16 maps) as a plain world and as a virtual strip, and the
# launch-cost / hipGraph lab. Every GPU step under its own time limit, chained with &&.
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread \
    -k "torch_conv_oracle or molecule_totals or payload or as_many" > $O/tests_new.log 2>&1 &&
timeout -k 10 300 python -u bench.py --map-size 5793 --cells 125000 --map-dtype fp16 > $O/m1share_plain.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 timeout -k 10 300 python -u bench.py --map-size 5793 --cells 125000 --map-dtype fp16 > $O/m1share_virtual.log 2>&1 &&
timeout -k 10 120 hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/lab/launch_lab.hip -o /tmp/launch_lab.bin &&
timeout -k 10 120 /tmp/launch_lab.bin > $O/launch_lab.log 2>&1
