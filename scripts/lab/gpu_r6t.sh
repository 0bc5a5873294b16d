#!/bin/bash
# Round 6, batch T: integrator latency floor -- one integrate (3 parts, 4 iterations, explicit X) on
# 200 / 2000 / 6250 / 50000 cells, and a kernel trace of the 200- and 6250-cell cases.
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python -u scripts/lab/ab_so.py --size 64 --cells 200 magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/int_200.log 2>&1 &&
timeout -k 10 120 python -u scripts/lab/ab_so.py --size 256 --cells 2000 magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/int_2000.log 2>&1 &&
timeout -k 10 120 python -u scripts/lab/ab_so.py --size 1448 --cells 6250 magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/int_6250.log 2>&1 &&
timeout -k 10 200 python -u scripts/lab/ab_so.py magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/int_50000.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt200 -o run --output-format csv -- python3 scripts/lab/ab_so.py --size 64 --cells 200 magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/kt200.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt6250 -o run --output-format csv -- python3 scripts/lab/ab_so.py --size 1448 --cells 6250 magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so > $O/kt6250.log 2>&1
