#!/bin/bash
# Round-4 GPU driver: gpu_r4.sh <outdir> <step>...  Steps: tests (maxfail 5), smoke, flagship, drv,
# proxy, virt, hsf, hsp, hsv, check, m1, wide, c1024, c256, tflag (kernel trace). Each GPU step has
# its own time limit; a fatal exit (timeout, abort, segfault) ends the script.
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
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.log"; fi
  if fatal $rc; then echo "fatal rc=$rc in $name"; tail -30 "$O/$name.log"; exit $rc; fi
  return 0
}
trace() {  # trace <name> <steps-to-summarise> <bench args...>
  local name="$1" k="$2"; shift 2
  echo "== trace $name $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python bench.py "$@" \
    > $O/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  if fatal $rc; then echo "fatal rc=$rc in $name"; tail -30 "$O/$name.log"; exit $rc; fi
  MARKER=${MARKER:-void msd::diffuse_stencil4} python scripts/lab/step_kernels.py $O/$name/run_kernel_trace.csv $k > $O/${name}_steps.txt 2>&1
}
for s in "$@"; do case "$s" in
  tests) run tests 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread ;;
  smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  flagship) run flagship 300 python bench.py ;;
  flagship2) run flagship2 300 python bench.py ;;
  drv) run drv 300 python bench.py --steps 20 --warmup 5 ;;
  proxy) run proxy8_plain 300 python bench.py --map-size 1448 --cells 6250 ;;
  virt) MS_VIRTUAL_STRIPS=1 run proxy8_virtual 300 python bench.py --map-size 1448 --cells 6250 ;;
  fvirt) MS_VIRTUAL_STRIPS=1 run flagship_virtual 300 python bench.py ;;
  hsf) run host_split_flagship 300 python scripts/lab/host_split.py 4096 50000 40 ;;
  hsp) run host_split_proxy8 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hsv) MS_VIRTUAL_STRIPS=1 run host_split_proxy8_virtual 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hspn) MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_proxy8_detail 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hsvn) MS_VIRTUAL_STRIPS=1 MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_proxy8_virtual_detail 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hspc) MS_CPROFILE=1 run host_split_proxy8_cprofile 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hsvc) MS_VIRTUAL_STRIPS=1 MS_CPROFILE=1 run host_split_proxy8_virtual_cprofile 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  upd) PROBE_PROFILE=1 run update_cells_probe 300 python scripts/lab/update_cells_probe.py ;;
  isweep) run integrator_sweep 300 python scripts/lab/integrator_sweep.py ;;
  dbench) run diffuse_bench 300 python scripts/lab/diffuse_bench.py --dtypes fp32 --blocks 1024 2048 0 --band 0 64 ;;
  iab) for i in 1 2; do for m in 0 4096; do MS_INTEGRATE_MODE=$m run iab_${m}_$i 300 python bench.py --steps 60 --warmup 20; done; done ;;
  wab) for i in 1 2; do for b in 64 128 256; do MS_FUSED_WIDE_BLOCKS=$b run wab_${b}_$i 300 python bench.py --steps 60 --warmup 20; done; done
       for b in 64 256; do MS_FUSED_WIDE_BLOCKS=$b run wsweep_$b 300 python scripts/lab/integrator_sweep.py 44000 50000 54000 60000; done ;;
  tcheck) echo "== trace tcheck"; timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/tcheck -o run --output-format csv -- python performance/check.py --parts update_cells > $O/tcheck.log 2>&1; echo "   rc=$?" ;;
  sab) for i in 1 2; do for w in 4 3 2; do MS_SPL2_WAVES=$w run sab_${w}_$i 300 python bench.py --preset wide --steps 40 --warmup 10; done; done ;;
  pmcw|pmcf) # PMC of the integrator / stencil kernels (one pass, 8 SQ counters, kernel filter, no trace domains)
     preset=$([ "$s" = pmcw ] && echo wide || echo flagship)
     echo "== pmc $preset"
     (cd /tmp && timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
        --kernel-include-regex "integrate|diffuse_stencil" -d "$OLDPWD/$O/pmc_$preset" -o run --output-format csv \
        -- python3 "$OLDPWD/bench.py" --preset $preset --steps 3 --warmup 2 > "$OLDPWD/$O/pmc_$preset.log" 2>&1)
     rc=$?; echo "   rc=$rc"; if fatal $rc; then exit $rc; fi ;;
  tcheck2) MS_TRANSLATE_TIMES=1 run check_translate 300 python performance/check.py --parts update_cells ;;
  tprobe) run translate_probe 300 python scripts/lab/translate_probe.py ;;
  checkp) MS_CHECK_PROFILE=1 run check_profile 600 python performance/check.py --parts update_cells mutations ;;
  check) run check 600 python performance/check.py ;;
  hbm) run hbm_bench 900 python bench.py --preset hbm --steps 10 --warmup 3 --step-times ;;
  m1) run m1_bench 600 python bench.py --preset m1 --steps 60 --warmup 10 --step-times ;;
  wide) run wide 300 python bench.py --preset wide ;;
  c1024) run c1024 300 python bench.py --preset c1024 --steps 30 --warmup 5 ;;
  c256) run c256_40k 300 python bench.py --map-size 256 --cells 40000 ;;
  tflag) trace tflag 19 --steps 20 --warmup 20 ;;
  tc256) trace tc256 19 --map-size 256 --cells 40000 --steps 20 --warmup 20 ;;
  hs256) MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_c256 300 python scripts/lab/host_split.py 256 40000 40 ;;
  hs256c) MS_CPROFILE=1 MS_CPROFILE_SORT=cumulative MS_CPROFILE_N=70 run host_split_c256_cprofile 300 python scripts/lab/host_split.py 256 40000 60 ;;
  twide) trace twide 19 --preset wide --steps 20 --warmup 20 ;;
  tlong) trace tlong 19 --steps 420 --warmup 20 ;;
  long500) run long500 600 python bench.py --steps 500 --warmup 20 --step-times ;;
  tm1) MARKER=_ZN3msd23diffuse_stencil8_kernel trace tm1 9 --preset m1 --steps 10 --warmup 5 ;;
  tfvirt) MARKER=msd::diffuse_corr_kernel MS_VIRTUAL_STRIPS=1 trace tfvirt 19 --steps 20 --warmup 20 ;;
  hsfv) MS_VIRTUAL_STRIPS=1 MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_flagship_virtual 300 python scripts/lab/host_split.py 4096 50000 40 ;;
  tpx) trace tpx 19 --map-size 1448 --cells 6250 --steps 20 --warmup 20 ;;
  tpxv) MARKER=msd::diffuse_corr_kernel MS_VIRTUAL_STRIPS=1 trace tpxv 19 --map-size 1448 --cells 6250 --steps 20 --warmup 20 ;;

  overlap) run overlap 300 python scripts/lab/overlap_probe.py 4096 50000 20 ;;
  *) echo "unknown step $s" ;;
esac; done
