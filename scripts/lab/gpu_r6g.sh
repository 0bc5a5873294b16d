#!/bin/bash
# Round 6, batch G: integrator argument blocks in device memory (fewer SGPR spills) -- in-process A/B
# against the previous build on the flagship and the wide chemistry, the GPU integrator tests, bench.
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "integrat or spec or register" > $O/int_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_so.py --steps 5 --iters 4 abx/base.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/ab_flagship.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_so.py --chem synthetic:64:256 --steps 5 --iters 4 abx/base.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/ab_wide.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
