#!/bin/bash
# Round 6, LONG2: how far an evolving flagship runs on the last tree -- 1000 timed steps after 5000
# evolving ones, and the proteome-shape probe over 8000 steps (scripts/lab/evo_shape.py).
# (the first try ran out of HBM before step 5000: a merged chain priced at 70 GB of scratch for a
# length bound of ~10^6 nt; calls now stay within genome_pipeline._BLOB_MAX and 1 GiB of slots)
set -o pipefail
O=$PWD/gpurun_out/r6long2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "genome_pipeline or merged or speculative or translation or param_build or huge or bench_steps or 8191" > $O/tests.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --steps 1000 --warmup 5000 > $O/flag_5000_1000.log 2>&1 || exit $?
timeout -k 10 500 python -u scripts/lab/evo_shape.py 8000 > $O/shape_8000.log 2>&1 || exit $?
