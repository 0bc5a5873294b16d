#!/bin/bash
# Round 6, batch E: kernel trace of the driver-style run (top-up spawn steps: the ragged parameter
# build) and the HBM preset's measured memory split.
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tdrv -o tdrv --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $O/tdrv.log 2>&1 &&
python3 scripts/lab/spawn_step.py $(ls $O/tdrv/*/tdrv_kernel_trace.csv $O/tdrv/tdrv_kernel_trace.csv 2>/dev/null | head -1) > $O/tdrv_spawn_steps.txt 2>&1 &&
timeout -k 10 400 python -u bench.py --preset hbm --steps 30 --warmup 10 > $O/hbm_bench.log 2>&1
