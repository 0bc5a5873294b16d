#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a ONE-GPU box: N ranks share cuda:0 and exchange over
# gloo (MS_DIST_BACKEND=gloo, device tensors staged through host copies), so DistributedWorld's strip
# kernels, halo / claim / migration exchanges and the bench's barrier+max-over-ranks timing run on the
# real device. RCCL itself (one rank per GPU) is exercised only by the driver's multi-GPU bench.
# usage: scripts/lab/gpu_dist_rehearsal.sh [ranks...]   (default: 2 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
export MS_DIST_BACKEND=gloo
ranks="${*:-2 4}"
port=29611
for n in $ranks; do
  echo "== ranks=$n" | tee -a gpurun_out/rehearsal.log
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus "$n" --steps 20 --warmup 10 \
    > "gpurun_out/rehearsal_$n.log" 2>&1
  rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/rehearsal.log
  grep '"metric"' "gpurun_out/rehearsal_$n.log" | tee -a gpurun_out/rehearsal.log
  [[ $rc -ne 0 ]] && { tail -20 "gpurun_out/rehearsal_$n.log"; exit $rc; }
  port=$((port + 1))
done
exit 0
