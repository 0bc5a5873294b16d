#!/bin/bash
# Round 6, batch Z: chunked LDS reads in the damping power loop -- in-process A/B against the tree
# before it (ab/int_base.so) at 200 / 6250 / 60000 cells and the wide chemistry.
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 120 python -u scripts/lab/ab_so.py --size 64 --cells 200 ab/int_base.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/ab_200.log 2>&1 &&
timeout -k 10 120 python -u scripts/lab/ab_so.py --size 1448 --cells 6250 ab/int_base.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/ab_6250.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_so.py ab/int_base.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/ab_flagship.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_so.py --chem synthetic:64:256 ab/int_base.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/ab_wide.log 2>&1
