#!/bin/bash
# rocprofv3 kernel stats of one bench config: scripts/gpu_profile_cfg.sh <name> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
export TMPDIR=/tmp
name="$1"; shift
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_$name -o run --output-format csv -- \
  python bench.py "$@" > gpurun_out/rocprof_$name.log 2>&1
rc=$?; echo "rocprof $name rc=$rc"; exit $rc
