#!/bin/bash
# Round 6, batch Q: driver-style runs (20 timed steps after 5 warmups) with per-step times and top-up
# counts, three times; the default bench once.
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --step-times > $O/drv_$i.log 2>&1 || exit $?
done
timeout -k 10 200 python -u bench.py > $O/flag.log 2>&1
