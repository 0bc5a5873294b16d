#!/bin/bash
# A/B of two source trees on one box: ab_base/ (a copy of an earlier commit with its own built
# extensions, git-ignored) against the working tree, alternating runs of the same bench command.
# usage: ab_trees.sh <outdir> <reps> <bench args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; reps=$2; shift 2
mkdir -p "$O"
for r in $(seq 1 "$reps"); do
  for t in base new; do
    if [ $t = base ]; then dir=ab_base; else dir=.; fi
    (cd $dir && PYTHONPATH="$PWD" timeout -k 10 300 python bench.py "$@") > "$O/${t}_$r.log" 2>&1
    rc=$?
    echo "$t rep $r rc=$rc $(grep -ho '"ms_per_step": [0-9.]*' "$O/${t}_$r.log")"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
