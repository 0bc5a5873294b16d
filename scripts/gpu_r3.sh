#!/bin/bash
# Round-3 GPU evidence driver: gpu_r3.sh <outdir> <step>...  Steps: tests, smoke, flagship, drv,
# check, proxy, virt, trace, c64, m1, c256, c1024. Every GPU step has its own time limit; a fatal
# exit (timeout, abort, segfault) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH="$PWD:${PYTHONPATH:-}" TMPDIR=/tmp
O=gpurun_out/$1; shift; rm -rf "$O"; mkdir -p "$O"
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # run <name> <seconds> <cmd...>
  local name="$1" secs="$2"; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc $(grep -h '^{"metric"' "$O/$name.log" | cut -c100-200)"
  if fatal $rc; then echo "fatal rc=$rc in $name"; tail -30 "$O/$name.log"; exit $rc; fi
  return 0
}
for s in "$@"; do case "$s" in
  tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
  smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  flagship) run flagship 300 python bench.py ;;
  drv) run drv 300 python bench.py --steps 20 --warmup 5 ;;
  check) run check 600 python performance/check.py ;;
  proxy) run proxy8_plain 300 python bench.py --map-size 1448 --cells 6250 ;;
  virt) MS_VIRTUAL_STRIPS=1 run proxy8_virtual 300 python bench.py --map-size 1448 --cells 6250 ;;
  fvirt) MS_VIRTUAL_STRIPS=1 run flagship_virtual 300 python bench.py ;;
  c64) run c4096_50k_64x256 400 python bench.py --chemistry synthetic:64:256 --steps 20 --warmup 5 ;;
  c256) run c256_40k 300 python bench.py --map-size 256 --cells 40000 ;;
  c1024) run c1024_10k_16x32_bf16 300 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --map-dtype bf16 --steps 30 --warmup 5 ;;
  m1) run c16384_1m_fp16 600 python bench.py --map-size 16384 --cells 1000000 --map-dtype fp16 --steps 50 --warmup 5 --step-times ;;
  hb) run host_breakdown 300 python scripts/host_breakdown.py 4096 50000 40 ;;
  hbv) MS_VIRTUAL_STRIPS=1 run host_breakdown_proxy8_virtual 300 python scripts/host_breakdown.py 1448 6250 60 ;;
  hbp) run host_breakdown_proxy8 300 python scripts/host_breakdown.py 1448 6250 60 ;;
  cpv) MS_VIRTUAL_STRIPS=1 run cprofile_proxy8_virtual 300 python scripts/step_cprofile.py 1448 6250 100 ;;
  cpp) run cprofile_proxy8 300 python scripts/step_cprofile.py 1448 6250 100 ;;
  wide) run wide_c4096_50k_64x256 300 python bench.py --preset wide ;;
  m1b) run m1_bench 600 python bench.py --preset m1 --steps 60 --warmup 10 --step-times ;;
  tproxy) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tproxy -o run --output-format csv -- \
            python bench.py --map-size 1448 --cells 6250 --steps 40 --warmup 20 > $O/tproxy.log 2>&1;
          python scripts/step_kernels.py $O/tproxy/run_kernel_trace.csv 39 > $O/tproxy_steps.txt 2>&1; echo "   traced" ;;
  tflag) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tflag -o run --output-format csv -- \
            python bench.py --steps 20 --warmup 20 > $O/tflag.log 2>&1;
          python scripts/step_kernels.py $O/tflag/run_kernel_trace.csv 19 > $O/tflag_steps.txt 2>&1; echo "   traced" ;;
  dbench) run diffuse_bench 300 python scripts/diffuse_bench.py --vec 4 8 --blocks 1024 0 2048 ;;
  dtests) run dtests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "diffusion or reduced_precision or permeation" ;;
  tc64) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tc64 -o run --output-format csv -- \
            python bench.py --chemistry synthetic:64:256 --steps 10 --warmup 5 > $O/tc64.log 2>&1;
          python scripts/step_kernels.py $O/tc64/run_kernel_trace.csv 9 > $O/tc64_steps.txt 2>&1; echo "   traced" ;;
  spk1m) MS_MAP_DTYPE=fp16 run spikes_1m 600 python scripts/spike_events.py 16384 1000000 40 5 ;;
  *) echo "unknown step $s"; exit 2 ;;
esac; done
exit 0
