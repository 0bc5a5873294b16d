#!/bin/bash
# Round 6, batch K: in-process A/B of the integrator argument blocks (ab/pre_args.so: kinetics.hip
# before c176d25) against the tree at the N = 8 proxy size and the flagship size.
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
S=magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so
timeout -k 10 300 python -u scripts/lab/ab_so.py --size 1448 --cells 6250 $S ab/pre_args.so > $O/ab_proxy.log 2>&1 &&
timeout -k 10 300 python -u scripts/lab/ab_so.py $S ab/pre_args.so > $O/ab_flagship.log 2>&1
