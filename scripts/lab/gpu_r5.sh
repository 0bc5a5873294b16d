#!/bin/bash
# Round-5 GPU driver: gpu_r5.sh <outdir> <step>...  Steps: tests (maxfail 5), smoke, flagship, drv,
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
  return $rc
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
  kt) run tests_kin 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "integrat or enzymatic or activity or kinetic" --timeout 300 --timeout-method thread ;;
  dt) run tests_diff 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -m gpu -q -x -k "diffus or stencil or mass or halo or strip" --timeout 300 --timeout-method thread ;;
  gt) run tests_gen 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_mutation_stats.py tests/test_gpu_distributed.py -m gpu -q -x -k "pipeline or recomb or evolve or merged or mutat or genetic" --timeout 300 --timeout-method thread ;;
  cbt) run tests_cb 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "chain_issued or pipeline or merged or recomb or kill_divide or lazy" --timeout 300 --timeout-method thread ;;
  selt) run tests_sel 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "select or kill_divide or chain_issued or lazy or placement or divide" --timeout 300 --timeout-method thread || exit 1 ;;
  selb) run select_bench 120 python scripts/lab/select_bench.py ;;
  ptab) for i in 1 2; do for t in 1 0; do MS_PLACE_TAIL=$t run ptab_${t}_$i 300 python bench.py; done; done ;;
  kab) for kn in ${KAB:-set_place_tail=1,0 set_select_single_pass=1,0}; do run kab_$(echo ${kn%%=*} | tr -c "a-zA-Z0-9_\n" _) 300 python scripts/lab/knob_ab.py $kn --blocks 10 --k 20; done ;;
  evlab) hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/lab/event_lab.hip -o /tmp/event_lab.bin && \
     (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d "$OLDPWD/$O/evlab" -o run --output-format csv -- /tmp/event_lab.bin) > $O/evlab.log 2>&1 && \
     python scripts/lab/event_lab_report.py $O/evlab/run_kernel_trace.csv | tee -a $O/evlab.log ;;
  virtab) for i in 1 2; do for c in 1,1 0,1 1,0 0,0; do IFS=, read pt ss <<< "$c"; MS_PLACE_TAIL=$pt MS_SELECT_SINGLE=$ss MS_VIRTUAL_STRIPS=1 run virtab_${pt}_${ss}_$i 300 python bench.py --map-size 1448 --cells 6250; done; done ;;
  cov) MS_VIRTUAL_STRIPS=1 run call_order_virtual 300 python scripts/lab/call_order.py 4096 50000 20 2 ;;
  kab256) for kn in ${KAB:-set_overflow_blocks=64,512}; do run kab256_$(echo ${kn%%=*} | tr -c "a-zA-Z0-9_\n" _) 300 python scripts/lab/knob_ab.py $kn --blocks 10 --k 20 --size 256 --cells 40000; done ;;
  co256) run call_order_c256 300 python scripts/lab/call_order.py 256 40000 20 3 ;;
  dcab) for i in 1 2; do for t in 1 0; do MS_DEVCOUNT_OPS=$t run dcab256_${t}_$i 300 python bench.py --map-size 256 --cells 40000; MS_DEVCOUNT_OPS=$t run dcabf_${t}_$i 300 python bench.py; done; done ;;
  lt) run tests_loop 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "deterministic or lazy or kill_divide or chain_issued or permeat or lifetime" --timeout 300 --timeout-method thread || exit 1 ;;
  spin) for i in 1 2; do for t in 1 0; do MS_EVENT_SPIN=$t run spin_${t}_$i 300 python bench.py; done; done ;;
  cbab) for i in 1 2 3; do for t in 1 0; do MS_CHAIN_BOUND=$t run cbab_${t}_$i 300 python bench.py; done; done ;;
  ssab) for i in 1 2; do for t in 1 0; do MS_SELECT_SINGLE=$t run ssab_${t}_$i 300 python bench.py; done; done ;;
  rthin) for i in 1 2; do for t in 1 0; do MS_REC_THIN=$t run rthin_${t}_$i 300 python bench.py; done; done ;;
  tmem) run tests_mem 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -k "memory_model or past_2_31" --timeout 300 --timeout-method thread ;;
  hipt) echo "== hipt $(date +%T)"; MS_VIRTUAL_STRIPS=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/hipt_virt -o run --output-format csv -- python bench.py --map-size 1448 --cells 6250 > $O/hipt_virt.log 2>&1; rc=$?; echo "   rc=$rc"; if fatal $rc; then exit $rc; fi ;;
  hiptp) echo "== hiptp $(date +%T)"; timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $O/hipt_plain -o run --output-format csv -- python bench.py --map-size 1448 --cells 6250 > $O/hipt_plain.log 2>&1; rc=$?; echo "   rc=$rc"; if fatal $rc; then exit $rc; fi ;;
  hsfv) MS_VIRTUAL_STRIPS=1 MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_flagship_virtual_detail 300 python scripts/lab/host_split.py 4096 50000 40 ;;
  stt) run tests_strip 600 python -u -m pytest tests/test_gpu_distributed.py -m gpu -q -x --timeout 300 --timeout-method thread ;;
  abearly) for i in 1 2; do for t in 1 0; do MS_EARLY_STENCIL=$t MS_VIRTUAL_STRIPS=1 run fvirt_e${t}_$i 300 python bench.py
            MS_EARLY_STENCIL=$t MS_VIRTUAL_STRIPS=1 run virt_e${t}_$i 300 python bench.py --map-size 1448 --cells 6250; done; done ;;
  tdrv) trace tdrv 19 --steps 20 --warmup 5 --step-times ;;
  splt) run tests_split 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_distributed.py -m gpu -q -x -k "place_split or strip or lazy" --timeout 300 --timeout-method thread ;;
  tests) run tests 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 120 --timeout-method thread ;;
  smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
  flagship) run flagship 300 python bench.py ;;
  flagship2) run flagship2 300 python bench.py ;;
  drv) run drv 300 python bench.py --steps 20 --warmup 5 ;;
  proxy) run proxy8_plain 300 python bench.py --map-size 1448 --cells 6250 ;;
  virt) MS_VIRTUAL_STRIPS=1 run proxy8_virtual 300 python bench.py --map-size 1448 --cells 6250 ;;
  fvirt) MS_VIRTUAL_STRIPS=1 run flagship_virtual 300 python bench.py ;;
  hsf) run host_split_flagship 300 python scripts/lab/host_split.py 4096 50000 40 ;;
  hsfc) MS_CPROFILE=1 MS_CPROFILE_SORT=cumulative MS_CPROFILE_N=80 run host_split_flagship_cprofile 300 python scripts/lab/host_split.py 4096 50000 40 ;;
  hsfn) MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_flagship_detail 300 python scripts/lab/host_split.py 4096 50000 40 ;;
  hsp) run host_split_proxy8 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hsv) MS_VIRTUAL_STRIPS=1 run host_split_proxy8_virtual 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hspn) MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_proxy8_detail 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hsvn) MS_VIRTUAL_STRIPS=1 MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_proxy8_virtual_detail 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hspc) MS_CPROFILE=1 run host_split_proxy8_cprofile 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  hsvc) MS_VIRTUAL_STRIPS=1 MS_CPROFILE=1 run host_split_proxy8_virtual_cprofile 300 python scripts/lab/host_split.py 1448 6250 60 ;;
  upd) PROBE_PROFILE=1 run update_cells_probe 300 python scripts/lab/update_cells_probe.py ;;
  isweep) run integrator_sweep 300 python scripts/lab/integrator_sweep.py ;;
  sab2) for i in 1 2; do for cfg in ${SAB2:-0,32,1024 2,64,768 2,64,512 3,64,512 1,64,768 2,64,1024 1,32,1024}; do IFS=, read pf bd bl <<< "$cfg"
         MS_STENCIL_PF=$pf MS_STENCIL_BAND=$bd MS_STENCIL_BLOCKS=$bl run sab2_${pf}_${bd}_${bl}_$i 300 python bench.py ${SAB2_ARGS:-}; done; done ;;
  dlab) for sk in 0 8192; do MS_MAP_SKEW=$sk run dlab_skew$sk 300 python scripts/lab/diffuse_bench.py --dtypes fp32 --pf 0 1 2 3 --band 0 64 --blocks 768 1024; done ;;
  dlab2) run dlab2 300 python scripts/lab/diffuse_bench.py --dtypes fp32 bf16 fp16 --pf 0 2 3 --band 0 64 --blocks 512 768 0 ;;
  dbench) run diffuse_bench 300 python scripts/lab/diffuse_bench.py --dtypes fp32 --blocks 1024 2048 0 --band 0 64 ;;
  iab) for i in 1 2; do for m in 0 4096; do MS_INTEGRATE_MODE=$m run iab_${m}_$i 300 python bench.py --steps 60 --warmup 20; done; done ;;
  abf) run ab_flagship 300 python scripts/lab/ab_so.py ${ABSO:-abso/head.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so}
       run ab_flagship_grown 300 python scripts/lab/ab_so.py --steps 150 ${ABSO:-abso/head.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so} ;;
  itc) for it in 0 1 2 4; do run itc_$it 300 python scripts/lab/ab_so.py --iters $it magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so; done ;;
  abw) run ab_wide 300 python scripts/lab/ab_so.py --chem synthetic:64:256 ${ABSO:-abso/head.so magicsoup_amd/_hip.cpython-310-x86_64-linux-gnu.so} ;;
  pmcst) # HBM bytes of the stencil (FETCH_SIZE: 3 TCC counters, WRITE_SIZE: 2 -> two passes)
     for c in FETCH_SIZE WRITE_SIZE; do
       (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "diffuse_stencil" -d "$OLDPWD/$O/pmc_stencil_$c" -o run --output-format csv \
          -- python3 "$OLDPWD/scripts/lab/diffuse_bench.py" --dtypes fp32 --iters 5 > "$OLDPWD/$O/pmc_stencil_$c.log" 2>&1)
       rc=$?; echo "   pmc $c rc=$rc"; if fatal $rc; then exit $rc; fi
     done ;;
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
  hbm) run hbm_bench 900 python bench.py --preset hbm --steps 60 --warmup 20 --step-times ;;
  m1) run m1_bench 600 python bench.py --preset m1 --steps 60 --warmup 10 --step-times ;;
  wide) run wide 300 python bench.py --preset wide ;;
  c1024) run c1024 300 python bench.py --preset c1024 --steps 30 --warmup 5 ;;
  c256) run c256_40k 300 python bench.py --map-size 256 --cells 40000 ;;
  tdrv) trace tdrv 19 --steps 20 --warmup 5 ;;
  hsdrv) MS_NATIVE_TIMES=1 MS_PY_TIMES=1 run host_split_drv 300 python scripts/lab/host_split.py 4096 50000 20 5 ;;
  drvst) run drv_step_times 300 python bench.py --steps 20 --warmup 5 --step-times ;;
  rsab) for i in 1 2 3; do for t in 1 0; do MS_BENCH_RESERVE=$t run rsab_${t}_$i 300 python bench.py --steps 20 --warmup 5 --step-times; done; done ;;
  drvst3) for i in 1 2 3; do run drv_step_times_$i 300 python bench.py --steps 20 --warmup 5 --step-times; done; run flag_step_times 300 python bench.py --step-times ;;
  poolt) run tests_pool 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "pool or spawn or arena or genome" --timeout 300 --timeout-method thread || exit 1 ;;
  smallab) for i in 1 2; do run c1024_$i 300 python bench.py --preset c1024 --steps 30 --warmup 5; run c256_$i 300 python bench.py --map-size 256 --cells 40000; done ;;
  c1024ab) run c1024_base 300 python bench.py --preset c1024 --steps 30 --warmup 5
     MS_SELECT_SINGLE=0 run c1024_sel0 300 python bench.py --preset c1024 --steps 30 --warmup 5
     MS_PLACE_TAIL=0 run c1024_tail0 300 python bench.py --preset c1024 --steps 30 --warmup 5
     MS_CHAIN_BOUND=1 run c1024_cb1 300 python bench.py --preset c1024 --steps 30 --warmup 5
     run c1024_base2 300 python bench.py --preset c1024 --steps 30 --warmup 5 ;;
  smallab2) for i in 1 2; do run c1024_$i 300 python bench.py --preset c1024 --steps 30 --warmup 5; run c256_$i 300 python bench.py --map-size 256 --cells 40000; run proxy_$i 300 python bench.py --map-size 1448 --cells 6250; done ;;
  tflag) trace tflag 19 --steps 20 --warmup 20 ;;
  tnodefer) MS_DEFER_GENOME_OPS=0 trace tnodefer 19 --steps 20 --warmup 20 ;;
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

  evolved) run evolved 600 python scripts/lab/evolved_probe.py --steps 500 --every 50 --modes 128 ;;
  sustained) run sustained 600 python bench.py --sustained --steps 200 --warmup 200 ;;
  overlap) run overlap 300 python scripts/lab/overlap_probe.py 4096 50000 20 ;;
  *) echo "unknown step $s" ;;
esac; done
