#!/bin/bash
# Run a list of bench.py configurations back to back on the GPU box, one JSON line per run in
# gpurun_out/matrix.jsonl (label prepended). Each run has its own time limit; a crash, abort or
# timeout stops the script.
# usage: scripts/lab/gpu_bench_matrix.sh "label|ENV=.. ENV2=..|bench args" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONPATH="$PWD:${PYTHONPATH:-}"
python -c "import __graft_entry__ as g; g.build()" || exit 1
for spec in "$@"; do
  IFS='|' read -r label envs args <<< "$spec"
  echo "== $label: $envs python bench.py $args"
  env $envs timeout -k 10 300 python bench.py $args > "gpurun_out/m_$label.log" 2> "gpurun_out/m_$label.err"
  rc=$?
  line=$(grep '^{"metric"' "gpurun_out/m_$label.log" || true)
  echo "{\"label\": \"$label\", \"env\": \"$envs\", \"args\": \"$args\", \"rc\": $rc, \"out\": ${line:-null}}" >> gpurun_out/matrix.jsonl
  echo "   rc=$rc ${line:0:200}"
  case $rc in 124|134|137|139) echo "fatal rc=$rc"; exit $rc;; esac
done
