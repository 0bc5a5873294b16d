#!/bin/bash
# Round 6, final matrix on the last tree: GPU suite, smoke, flagship, driver-style, per-rank proxies
# (plain / virtual strip), flagship as one strip, 256^2 / 40k, c1024, wide, m1, check.py.
# usage: bash scripts/lab/gpu_r6final.sh A|B  (two calls: each stays within one gpurun limit)
set -o pipefail
O=gpurun_out/r6final
mkdir -p $O
run() {  # name seconds cmd...: a failing step is logged; a crash / timeout ends the script
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> $O/status.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
case "$1" in
A)
  run gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  run flag_1 200 python -u bench.py
  run drv_1 200 python -u bench.py --steps 20 --warmup 5
  run plain8_1 200 python -u bench.py --map-size 1448 --cells 6250
  MS_VIRTUAL_STRIPS=1 run virt8_1 200 python -u bench.py --map-size 1448 --cells 6250
  run flag_2 200 python -u bench.py
  run drv_2 200 python -u bench.py --steps 20 --warmup 5
  run plain8_2 200 python -u bench.py --map-size 1448 --cells 6250
  MS_VIRTUAL_STRIPS=1 run virt8_2 200 python -u bench.py --map-size 1448 --cells 6250
  ;;
B)
  MS_VIRTUAL_STRIPS=1 run flagvirt 200 python -u bench.py
  run c256 200 python -u bench.py --map-size 256 --cells 40000
  run c1024 200 python -u bench.py --preset c1024 --steps 30 --warmup 5
  run wide 300 python -u bench.py --preset wide
  run m1 600 python -u bench.py --preset m1 --steps 60 --warmup 10
  run check 600 python -u performance/check.py
  ;;
esac
