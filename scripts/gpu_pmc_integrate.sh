#!/bin/bash
# PMC counters of the integrator kernels at the flagship config (one counter pass per run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/pmc; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --kernel-include-regex integrate -d $O/p1 -o run --output-format csv -- python bench.py --steps 5 --warmup 5 > $O/p1.log 2>&1
echo "pass1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY --kernel-include-regex integrate -d $O/p2 -o run --output-format csv -- python bench.py --steps 5 --warmup 5 > $O/p2.log 2>&1
echo "pass2 rc=$?"
find $O -name "*counter_collection.csv" | head
exit 0
