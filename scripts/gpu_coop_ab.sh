#!/bin/bash
# Cooperative placement kernel time vs its workgroup count (MS_COOP_BLOCKS), from rocprofv3 stats
# of the flagship bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
for b in 64 128 256 512; do
  rm -rf gpurun_out/coop$b
  MS_COOP_BLOCKS=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/coop$b -o run --output-format csv -- python bench.py --steps 20 --warmup 10 > gpurun_out/coop$b.log 2>&1
  echo "blocks $b: $(grep -h place_rounds_coop gpurun_out/coop$b/run_kernel_stats.csv | cut -d, -f1-5)"
done
exit 0
