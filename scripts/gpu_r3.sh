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
trace() {  # trace <name> <steps-to-summarise> <bench args...>: kernel trace + --stats of a bench run
  local name="$1" k="$2"; shift 2
  echo "== trace $name $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python bench.py "$@" \
    > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc $(grep -h '^{"metric"' "$O/$name.log" | cut -c100-200)"
  if fatal $rc; then echo "fatal rc=$rc in $name"; tail -30 "$O/$name.log"; exit $rc; fi
  python scripts/step_kernels.py $O/$name/run_kernel_trace.csv $k > $O/${name}_steps.txt 2>&1
}
htrace() {  # htrace <name> <steps> <bench args...>: HIP API + kernel trace, host / device timeline of a bench run
  local name="$1" k="$2"; shift 2
  echo "== htrace $name $(date +%T)"
  timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d $O/$name -o run --output-format csv -- python bench.py "$@" \
    > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  if fatal $rc; then echo "fatal rc=$rc in $name"; tail -30 "$O/$name.log"; exit $rc; fi
  python scripts/host_timeline.py $O/$name $k > $O/${name}_host.txt 2>&1
  rm -f $O/$name/run_hip_api_trace.csv
}
pmc() {  # pmc <name> <kernel regex> <counters> -- <bench args...>: one counter pass (no tracing domains)
  local name="$1" kr="$2" ctr="$3"; shift 4
  echo "== pmc $name $(date +%T)"
  timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-include-regex "$kr" -d $O/$name -o run --output-format csv -- \
    python bench.py "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  if fatal $rc; then echo "fatal rc=$rc in $name"; tail -30 "$O/$name.log"; exit $rc; fi
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
  c1024f) run c1024_10k_16x32_fp32 300 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --map-dtype fp32 --steps 30 --warmup 5 ;;
  c1024) run c1024_10k_16x32_bf16 300 python bench.py --map-size 1024 --cells 10000 --chemistry synthetic:16:32 --map-dtype bf16 --steps 30 --warmup 5 ;;
  m1) run c16384_1m_fp16 600 python bench.py --map-size 16384 --cells 1000000 --map-dtype fp16 --steps 50 --warmup 5 --step-times ;;
  hb) run host_breakdown 300 python scripts/host_breakdown.py 4096 50000 40 ;;
  hbv) MS_VIRTUAL_STRIPS=1 run host_breakdown_proxy8_virtual 300 python scripts/host_breakdown.py 1448 6250 60 ;;
  hbp) run host_breakdown_proxy8 300 python scripts/host_breakdown.py 1448 6250 60 ;;
  hsv) MS_VIRTUAL_STRIPS=1 run host_split_proxy8_virtual 300 python scripts/host_split.py 1448 6250 60 ;;
  hsp) run host_split_proxy8 300 python scripts/host_split.py 1448 6250 60 ;;
  hsn) MS_NATIVE_TIMES=1 MS_VIRTUAL_STRIPS=1 run host_native_proxy8_virtual 300 python scripts/host_split.py 1448 6250 60 ;;
  hsnp) MS_NATIVE_TIMES=1 run host_native_proxy8 300 python scripts/host_split.py 1448 6250 60 ;;
  hspy) MS_PY_TIMES=1 MS_NATIVE_TIMES=1 run host_py_proxy8 300 python scripts/host_split.py 1448 6250 60 ;;
  hspyv) MS_PY_TIMES=1 MS_NATIVE_TIMES=1 MS_VIRTUAL_STRIPS=1 run host_py_proxy8_virtual 300 python scripts/host_split.py 1448 6250 60 ;;
  hsf) run host_split_flagship 300 python scripts/host_split.py 4096 50000 40 ;;
  cpv) MS_VIRTUAL_STRIPS=1 run cprofile_proxy8_virtual 300 python scripts/step_cprofile.py 1448 6250 100 ;;
  cpvc) MS_PROF_LINES=90 MS_VIRTUAL_STRIPS=1 run cprofile_proxy8_virtual_cum 300 python scripts/step_cprofile.py 1448 6250 100 cumulative ;;
  cpvn) MS_PROF_LINES=60 MS_VIRTUAL_STRIPS=1 run cprofile_proxy8_virtual_ncalls 300 python scripts/step_cprofile.py 1448 6250 100 ncalls ;;
  cpp) run cprofile_proxy8 300 python scripts/step_cprofile.py 1448 6250 100 ;;
  cppc) MS_PROF_LINES=90 run cprofile_proxy8_cum 300 python scripts/step_cprofile.py 1448 6250 100 cumulative ;;
  wide) run wide_c4096_50k_64x256 300 python bench.py --preset wide ;;
  m1b) run m1_bench 600 python bench.py --preset m1 --steps 60 --warmup 10 --step-times ;;
  tproxy) trace tproxy 39 --map-size 1448 --cells 6250 --steps 40 --warmup 20 ;;
  tvirt) MS_VIRTUAL_STRIPS=1 trace tvirt 39 --map-size 1448 --cells 6250 --steps 40 --warmup 20 ;;
  tflag) trace tflag 19 --steps 20 --warmup 20 ;;
  tfvirt) MS_VIRTUAL_STRIPS=1 trace tfvirt 19 --steps 20 --warmup 20 ;;
  hsfv) MS_PY_TIMES=1 MS_NATIVE_TIMES=1 MS_VIRTUAL_STRIPS=1 run host_py_flagship_virtual 300 python scripts/host_split.py 4096 50000 40 ;;
  htflag) htrace htflag 10 --steps 12 --warmup 20 ;;
  htproxy) htrace htproxy 10 --map-size 1448 --cells 6250 --steps 12 --warmup 20 ;;
  tenv) timeout -k 10 120 rocprofv3 --kernel-trace -d $O/tenv -o run --output-format csv -- python -c "import os; print(sorted(k for k in os.environ if 'ROC' in k))" > $O/tenv.log 2>&1; echo "   rc=$?" ;;
  dbench) run diffuse_bench 300 python scripts/diffuse_bench.py --vec 4 8 --blocks 1024 0 2048 ;;
  dbband) run diffuse_bench_band 400 python scripts/diffuse_bench.py --vec 0 --blocks 1024 2048 --band 16 32 48 64 --dtypes fp32 fp16 && run diffuse_bench_band64 400 python scripts/diffuse_bench.py --chem synthetic:64:256 --vec 0 --blocks 1024 2048 --band 16 32 64 --dtypes fp32 --iters 10 ;;
  dbpf) run diffuse_bench_pf 300 python scripts/diffuse_bench.py --vec 4 8 --blocks 1024 2048 --pf 0 1 2 3 ;;
  dtests) run dtests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "diffusion or reduced_precision or permeation" ;;
  dbauto) run diffuse_bench_auto 400 python scripts/diffuse_bench.py --vec 0 --blocks 1024 --band 0 32 --dtypes fp32 fp16 && run diffuse_bench_auto64 400 python scripts/diffuse_bench.py --chem synthetic:64:256 --vec 0 --blocks 1024 --band 0 32 --dtypes fp32 --iters 10 ;;
  tc64) trace tc64 9 --preset wide --steps 10 --warmup 5 ;;
  tm1) trace tm1 19 --preset m1 --steps 20 --warmup 10 ;;
  pmcw1) pmc pmc_wide_sq "integrate|gather_bin|diffuse_stencil" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" -- --preset wide --steps 3 --warmup 3 ;;
  pmcw2) pmc pmc_wide_fetch "integrate|diffuse_stencil" "FETCH_SIZE" -- --preset wide --steps 3 --warmup 3 ;;
  pmcw3) pmc pmc_wide_write "integrate|diffuse_stencil" "WRITE_SIZE" -- --preset wide --steps 3 --warmup 3 ;;
  spk1m) MS_MAP_DTYPE=fp16 run spikes_1m 600 python scripts/spike_events.py 16384 1000000 70 10 ;;
  spk1mw) MS_GENOME_WIDTH_WATCH=1 MS_MAP_DTYPE=fp16 run spikes_1m_watch 600 python scripts/spike_events.py 16384 1000000 70 10 ;;
  *) echo "unknown step $s"; exit 2 ;;
esac; done
exit 0
