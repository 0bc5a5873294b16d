#!/bin/bash
# The reference's performance workloads (performance/check.py, performance/run_simulation.py) plus the
# flagship bench (bench.py) on the current device.
set -euo pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
python -m magicsoup_amd.ops.build
python performance/check.py "$@"
python performance/run_simulation.py --n-steps 200
python bench.py
