#!/bin/bash
# Stencil A/B of two builds on one box: gpu_stencil_ab.sh <outdir> <old.so>. Diffusion tests with the
# in-tree build, then diffuse_bench + flagship benches alternating the in-tree build (new) and <old.so>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/$1; OLD=$2; rm -rf "$O"; mkdir -p "$O"
SO=magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/new.so
run() {  # run <name> <seconds> <cmd...>; stops the script on a failure
  local name="$1" secs="$2"; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc $(grep -h '^{"metric"' "$O/$name.log" | cut -c100-200)"
  if [ $rc -ne 0 ]; then tail -20 "$O/$name.log"; cp /tmp/new.so $SO; exit $rc; fi
}
run tests_diff 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -m gpu -q -x -k "diffus or stencil or mass or halo or strip" --timeout 300 --timeout-method thread
for i in 1 2; do
  for v in new old; do
    if [ $v = new ]; then cp /tmp/new.so $SO; else cp $OLD $SO; fi
    run dbench_${v}_$i 300 python scripts/lab/diffuse_bench.py --dtypes fp32 bf16 --vec 4 8 --blocks 512 768
    run flagship_${v}_$i 300 python bench.py
  done
done
cp /tmp/new.so $SO
