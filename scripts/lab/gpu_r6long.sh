#!/bin/bash
# Round 6, batch LONG: longevity of the last tree (ragged records, pool collections, deterministic
# spawns over many evolving steps): flagship 3000 steps, 256^2 / 40k 3000 steps, the N = 8 virtual
# strip 2000 steps, m1 300 steps, the HBM preset 100 steps.
set -o pipefail
O=gpurun_out/r6long
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 3000 --warmup 20 > $O/flag3000.log 2>&1 &&
timeout -k 10 300 python -u bench.py --map-size 256 --cells 40000 --steps 3000 --warmup 20 > $O/c256_3000.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 timeout -k 10 300 python -u bench.py --map-size 1448 --cells 6250 --steps 2000 --warmup 20 > $O/virt8_2000.log 2>&1 &&
timeout -k 10 300 python -u bench.py --preset m1 --steps 300 --warmup 10 > $O/m1_300.log 2>&1 &&
timeout -k 10 600 python -u bench.py --preset hbm --steps 100 --warmup 5 > $O/hbm_100.log 2>&1
