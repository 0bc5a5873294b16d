#!/bin/bash
# Second PMC group (instruction mix, LDS bank conflicts) over the integrator kernels (see
# gpu_integrator_pmc.sh; rocprofv3 may segfault at teardown after writing its CSV).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipmc
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
REPO="$PWD"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT \
  --kernel-include-regex "integrate" -d "$REPO/gpurun_out/ipmc/g2_4096" -o run --output-format csv -- \
  python3 "$REPO/scripts/integrator_pmc.py" 4096 50000 3 > "$REPO/gpurun_out/ipmc/g2_4096.log" 2>&1
echo "rc=$?"
exit 0
