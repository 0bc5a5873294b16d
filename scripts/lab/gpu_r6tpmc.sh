#!/bin/bash
# Round 6, TPMC: counters of the long-genome translation pass (scripts/lab/tlong_bench.py), one pass
# per counter group: where a workgroup's time goes for a 200k-nt genome.
set -o pipefail
O=$PWD/gpurun_out/r6tpmc
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY -d $O/sq -o run --output-format csv -- python3 scripts/lab/tlong_bench.py > $O/sq.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o run --output-format csv -- python3 scripts/lab/tlong_bench.py > $O/tcc.log 2>&1 || exit $?
