#!/bin/bash
# Round 6, batch I: host split of the N = 8 proxy (1448^2 / 6250) as a virtual strip and plain:
# per-op busy / blocked host time, native entry points, and a cProfile of the virtual strip step.
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
MS_VIRTUAL_STRIPS=1 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hs_virtual.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 MS_NATIVE_TIMES=1 MS_PY_TIMES=1 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hs_virtual_detail.log 2>&1 &&
MS_NATIVE_TIMES=1 MS_PY_TIMES=1 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hs_plain_detail.log 2>&1 &&
MS_VIRTUAL_STRIPS=1 MS_CPROFILE=1 MS_CPROFILE_SORT=tottime MS_CPROFILE_N=60 timeout -k 10 200 python -u scripts/lab/host_split.py 1448 6250 60 > $O/hs_virtual_cprofile.log 2>&1
