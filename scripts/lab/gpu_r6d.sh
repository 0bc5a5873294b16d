#!/bin/bash
# Round 6, batch D: HBM-filling worlds on ragged parameter records -- the planned preset (the map
# now takes the memory the dense parameter rows held) and round 5's widen config (37632^2 / 5.3M
# cells, which died widening its dense rows) for 100 evolving steps.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 500 python -u bench.py --preset hbm --steps 60 --warmup 20 --step-times > $O/hbm_bench.log 2>&1 &&
timeout -k 10 500 python -u bench.py --preset hbm --map-size 37632 --cells 5275634 --steps 100 --warmup 5 --memory-report > $O/hbm_widen.log 2>&1
