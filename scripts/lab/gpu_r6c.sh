#!/bin/bash
# Round 6, batch C: the rest of the GPU suite after test_ragged_records_match_host_build, the bench,
# the HBM-filling preset (ragged records: planned map size) and the widen config of round 5.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    --deselect tests/test_gpu_kernels.py::test_merged_recombinate_mutate_chain_matches_separate_calls > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 60 --warmup 20 > $O/bench2.log 2>&1
