#!/bin/bash
# Host (cProfile) and device (rocprofv3 kernel stats) profiles of the flagship step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
export TMPDIR=/tmp
MAP="${1:-256}"; CELLS="${2:-40000}"
python -c "import __graft_entry__ as g; g.build()" || exit 1
timeout -k 10 300 python scripts/profile_step.py "$MAP" "$CELLS" 10 > gpurun_out/cprofile_${MAP}.log 2>&1
rc=$?; echo "cprofile rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_${MAP} -o run --output-format csv -- \
  python bench.py --map-size "$MAP" --cells "$CELLS" --steps 10 --warmup 10 > gpurun_out/rocprof_bench_${MAP}.log 2>&1
rc=$?; echo "rocprof rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
# phase-attributed trace: roctx ranges around every World op + device drained at phase boundaries
MS_ROCTX=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/prof_${MAP}_phases -o run \
  --output-format csv -- python bench.py --map-size "$MAP" --cells "$CELLS" --steps 10 --warmup 10 \
  --profile-phases --phase-sync > gpurun_out/rocprof_phases_${MAP}.log 2>&1
rc=$?; echo "rocprof phases rc=$rc"
find gpurun_out/prof_${MAP}* -name "*.csv" | head -20
