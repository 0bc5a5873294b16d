#!/bin/bash
# Per-rank cost of the strong-scaling flagship on ONE GPU: a single world with 1/N of the 4096^2
# pixels and 1/N of the 50k cells approximates one rank's compute at N GPUs (no communication).
# Then a kernel trace of the N=8 share (launches / kernel-busy / idle per step).
# usage: scripts/gpu_rank_share.sh [trace]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
export TMPDIR=/tmp
mode="${1:-}"
python -c "import __graft_entry__ as g; g.build()" || exit 1
for cfg in "4096 50000 1" "2896 25000 2" "2048 12500 4" "1448 6250 8"; do
  [[ "$mode" == trace-only ]] && break
  set -- $cfg
  timeout -k 10 300 python bench.py --map-size "$1" --cells "$2" --steps 100 --warmup 20 \
    > "gpurun_out/share_$3.log" 2>&1
  rc=$?
  echo "share N=$3 rc=$rc $(grep '"metric"' gpurun_out/share_$3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step")')"
  case $rc in 0) ;; *) tail -5 "gpurun_out/share_$3.log"; exit $rc;; esac
done
if [[ "$mode" == trace* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_share8 -o run --output-format csv -- \
    python bench.py --map-size 1448 --cells 6250 --steps 20 --warmup 20 > gpurun_out/prof_share8.log 2>&1
  rc=$?; echo "trace rc=$rc"
  f=$(find gpurun_out/prof_share8 -name "*kernel_trace.csv" | head -1)
  [[ -n "$f" ]] && python scripts/trace_summary.py "$f" 20 --per-step 6 > gpurun_out/trace_share8.txt
  [[ -n "$f" ]] && python scripts/gap_summary.py "$f" > gpurun_out/gaps_share8.txt
  timeout -k 10 300 python bench.py --map-size 1448 --cells 6250 --steps 50 --warmup 20 --profile-phases \
    > gpurun_out/phases_share8.log 2>&1
  echo "phases rc=$?"
fi
exit 0
