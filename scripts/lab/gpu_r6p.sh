#!/bin/bash
# Round 6, batch P: GPU suite (per-op exact 2-rank physics, native cell decay / lifetimes), flagship
# and N = 8 proxies.
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
true
timeout -k 10 200 python -u scripts/lab/param_paths.py 30000 > $O/param_paths_30k.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > $O/flag.log 2>&1 &&
timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/plain8.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/virt8.log 2>&1
