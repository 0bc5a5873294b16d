#!/bin/bash
# PMC passes (one per counter group, kernel trace only) over the integrator kernels, both launch
# modes (scripts/lab/integrator_pmc.py).  usage: scripts/lab/gpu_integrator_pmc.sh [map_size cells]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ipmc
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
REPO="$PWD"
python -c "import __graft_entry__ as g; g.build()" || exit 1
cd /tmp && export TMPDIR=/tmp
S="${1:-4096}"; C="${2:-50000}"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "integrate" -d "$REPO/gpurun_out/ipmc/g${i}_$S" -o run \
    --output-format csv -- python3 "$REPO/scripts/lab/integrator_pmc.py" "$S" "$C" 3 > "$REPO/gpurun_out/ipmc/g${i}_$S.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  case $rc in 0) ;; *) tail -5 "$REPO/gpurun_out/ipmc/g${i}_$S.log"; exit $rc;; esac
done
