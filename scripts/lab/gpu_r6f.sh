#!/bin/bash
# Round 6, batch F: deterministic spawn placement (priority-round claims): the spawn tests first,
# then the GPU suite and the bench.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "spawn or deterministic" > $O/spawn_tests.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/drv.log 2>&1
