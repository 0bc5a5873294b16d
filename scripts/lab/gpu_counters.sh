#!/bin/bash
# PMC counters for the hot kernels (one rocprofv3 pass per counter group; no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
REPO="$PWD"
cd /tmp && export TMPDIR=/tmp
KR="${KR:-integrate_part|diffuse_stencil|diffuse_correct|gather_rows}"
# PMC_GROUPS="1 2 4" selects groups by number (FETCH_SIZE = group 3 and WRITE_SIZE = group 6 each need
# a pass of their own: together they exceed the 4 TCC counters one pass can hold)
PMC_GROUPS="${PMC_GROUPS:-1 2 3 4 5 6}"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "OccupancyPercent MeanOccupancyPerActiveCU" "LDSBankConflict" "WRITE_SIZE"; do
  i=$((i+1))
  case " $PMC_GROUPS " in *" $i "*) ;; *) continue;; esac
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$KR" -d "$REPO/gpurun_out/pmc/g$i" -o run \
    --output-format csv -- python3 "$REPO/scripts/lab/kernel_bench.py" 4096 50000 3 > "$REPO/gpurun_out/pmc/g$i.log" 2>&1
  rc=$?; echo "group $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
