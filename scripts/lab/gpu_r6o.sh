#!/bin/bash
# Round 6, batch O: in-process A/B of graph-batched vs direct launches (alternating step blocks in one
# world): N = 8 proxy plain and virtual strip, the flagship, 256^2 / 40k.
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
timeout -k 10 300 python -u scripts/lab/ab_batch.py 1448 6250 10 20 > $O/ab_plain8.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 timeout -k 10 300 python -u scripts/lab/ab_batch.py 1448 6250 10 20 > $O/ab_virt8.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_batch.py 4096 50000 8 20 > $O/ab_flagship.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 timeout -k 10 300 python -u scripts/lab/ab_batch.py 4096 50000 8 20 > $O/ab_flagship_virt.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_batch.py 256 40000 8 20 > $O/ab_c256.log 2>&1
