#!/bin/bash
# Round-2 closing evidence for profiles/: bench lines of every BASELINE config, the untraced step
# timeline / host breakdown / slow-step events of the flagship, the per-rank floor of an 8-GPU job
# (plain and as virtual strips), and a kernel trace + stats of the flagship step. Every GPU step
# has its own time limit; a fatal exit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/end; rm -rf $O; mkdir -p $O
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc $(grep -h '^{"metric"' "$O/$name.log" | cut -c100-190)"
  if fatal $rc; then echo "fatal rc=$rc in $name"; exit $rc; fi
  return 0
}
run flagship_a 300 python bench.py
run flagship_b 300 python bench.py
run flagship_drv 300 python bench.py --steps 20 --warmup 5
run c256_40k 300 python bench.py --map-size 256 --cells 40000
run c1024_10k_16x32_fp32 300 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --steps 30 --warmup 5
run c1024_10k_16x32_bf16 300 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --map-dtype bf16 --steps 30 --warmup 5
run c4096_50k_64x256 400 python bench.py --map-size 4096 --cells 50000 --chemistry synthetic:64:256 --steps 20 --warmup 5
run c16384_1m_fp16 600 python bench.py --map-size 16384 --cells 1000000 --map-dtype fp16 --steps 10 --warmup 3
run proxy8_plain 300 python bench.py --map-size 1448 --cells 6250
MS_VIRTUAL_STRIPS=1 run proxy8_virtual 300 python bench.py --map-size 1448 --cells 6250
MS_VIRTUAL_STRIPS=1 run flagship_virtual 300 python bench.py
run step_timeline 300 python scripts/step_timeline.py 4096 50000 40 p
run host_breakdown 300 python scripts/host_breakdown.py 4096 50000 40
MS_VIRTUAL_STRIPS=1 run host_breakdown_proxy8_virtual 300 python scripts/host_breakdown.py 1448 6250 60
run spike_events 300 python scripts/spike_events.py 4096 50000 100
# kernel trace + stats of the flagship step (rocprofv3 may crash at teardown after writing its
# output: its exit status is not checked)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python bench.py --steps 20 --warmup 20 > $O/trace.log 2>&1
python scripts/step_kernels.py $O/trace/run_kernel_trace.csv 19 > $O/step_kernels.txt 2>&1
ls $O/trace
exit 0
