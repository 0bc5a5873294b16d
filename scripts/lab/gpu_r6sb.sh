#!/bin/bash
# Round 6, batch SB: stencil grid size at the N = 8 proxy size (1448^2, 14 species fp32) -- plain and
# virtual-strip proxies with MS_STENCIL_BLOCKS 256 / 512 (default) / 1024, twice, interleaved.
set -o pipefail
O=gpurun_out/r6sb
mkdir -p $O
for i in 1 2; do
  for b in 512 1024 256; do
    MS_STENCIL_BLOCKS=$b timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/plain_b${b}_$i.log 2>&1 || exit $?
    MS_STENCIL_BLOCKS=$b MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u bench.py --map-size 1448 --cells 6250 > $O/virt_b${b}_$i.log 2>&1 || exit $?
  done
done
