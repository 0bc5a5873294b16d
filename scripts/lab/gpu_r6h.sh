#!/bin/bash
# Round 6, batch H: the N = 8 per-rank proxy (1448^2 / 6250 cells) as a plain world and as a
# virtual strip (the full strip protocol against itself over RCCL), twice each, plus a HIP API /
# kernel trace of the virtual strip (launches per step).
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/proxy8_plain_$i.log 2>&1 || exit $?
  MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/proxy8_virtual_$i.log 2>&1 || exit $?
done
MS_VIRTUAL_STRIPS=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/hipt_virt -o run --output-format csv -- python3 bench.py --map-size 1448 --cells 6250 > $O/hipt_virt.log 2>&1 &&
python3 scripts/lab/hip_api_per_step.py $(dirname $(ls $O/hipt_virt/*/run_kernel_trace.csv $O/hipt_virt/run_kernel_trace.csv 2>/dev/null | head -1)) > $O/hip_api_per_step_virtual.txt 2>&1
