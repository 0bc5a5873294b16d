#!/bin/bash
# A/B of two builds of the _hip extension on one box: gpu_so_ab.sh <outdir> <old.so> [pytest -k expr].
# GPU tests (selected by the -k expression) with the in-tree build, then driver-style, flagship and
# 1024^2 benches alternating the in-tree build (new) and <old.so>; the in-tree build is restored.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/$1; OLD=$2; K=${3:-param or pipeline or host_core or build}; rm -rf "$O"; mkdir -p "$O"
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
run tests 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "$K" --timeout 300 --timeout-method thread
for i in 1 2; do
  for v in new old; do
    if [ $v = new ]; then cp /tmp/new.so $SO; else cp $OLD $SO; fi
    run drv_${v}_$i 300 python bench.py --steps 20 --warmup 5 --step-times
    run flagship_${v}_$i 300 python bench.py
    run c1024_${v}_$i 300 python bench.py --preset c1024 --steps 30 --warmup 5
  done
done
cp /tmp/new.so $SO
