#!/bin/bash
# Round 6, batch B: the GPU suite and the flagship bench on the ragged parameter records.
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
