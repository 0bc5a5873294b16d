#!/bin/bash
# A/B of the early diffusion stencil's variants on the flagship bench (alternating, two rounds):
# off; issued after the kill's spill / after its compaction sync; deferred genome chains flushed at
# once or at the diffusion. Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/eab; rm -rf $O; mkdir -p $O
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for r in 1 2; do
  for v in "off:MS_EARLY_DIFFUSE=0" "spill_flush:MS_EARLY_DIFFUSE_AT=spill MS_FLUSH_EARLY=1" \
           "spill_late:MS_EARLY_DIFFUSE_AT=spill MS_FLUSH_EARLY=0" "synced_flush:MS_EARLY_DIFFUSE_AT=synced MS_FLUSH_EARLY=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 300 python bench.py > $O/$name.$r.log 2>&1
    rc=$?
    echo "$name.$r rc=$rc $(grep -h '^{"metric"' $O/$name.$r.log | cut -c100-175)"
    if fatal $rc; then exit $rc; fi
  done
done
MS_EARLY_DIFFUSE_AT=spill MS_FLUSH_EARLY=1 TS_OUT=$O/ts bash scripts/gpu_trace_step.sh > $O/trace_step.log 2>&1
exit 0
