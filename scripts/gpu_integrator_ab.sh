#!/bin/bash
# Integrator A/B on the GPU: kernel tests, then register-resident (mode 0) vs legacy LDS-staged
# (mode 8) launches on the same states at the flagship size and at one rank's share of 8 GPUs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
python -c "import __graft_entry__ as g; g.build()" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/ab_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab_pytest.log
case $rc in 0) ;; *) exit $rc;; esac
for cfg in "4096 50000" "1448 6250"; do
  set -- $cfg
  timeout -k 10 300 python scripts/integrator_bench.py "$1" "$2" > "gpurun_out/ab_$1.json" 2> "gpurun_out/ab_$1.err"
  rc=$?; echo "bench $1 rc=$rc"; cat "gpurun_out/ab_$1.json"
  case $rc in 0) ;; *) tail -5 "gpurun_out/ab_$1.err"; exit $rc;; esac
done
