#!/bin/bash
# In-process A/B of _hip builds (scripts/ab_so.py) at the flagship size and one rank's share of 8.
# usage: scripts/gpu_ab_so.sh A.so B.so [...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
python -c "import __graft_entry__ as g; g.build()" || exit 1
sos=("$@")
for cfg in "1448 6250" "4096 50000"; do
  set -- $cfg
  timeout -k 10 300 python scripts/ab_so.py --size "$1" --cells "$2" "${sos[@]}" > "gpurun_out/abso_$1.json" 2> "gpurun_out/abso_$1.err"
  rc=$?; echo "ab $1 rc=$rc"; cat "gpurun_out/abso_$1.json"
  case $rc in 0) ;; *) tail -5 "gpurun_out/abso_$1.err"; exit $rc;; esac
done
