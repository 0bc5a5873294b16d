#!/bin/bash
# A/B of environment settings on one box: alternating bench runs of the same tree.
# usage: ab_env.sh <outdir> <reps> "<env A>" "<env B>" ... -- <bench args...>
#   (an env spec is a space-separated list of VAR=value, "-" for none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; reps=$2; shift 2
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift
mkdir -p "$O"
for r in $(seq 1 "$reps"); do
  for i in "${!envs[@]}"; do
    e="${envs[$i]}"; [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py "$@" > "$O/v${i}_$r.log" 2>&1
    rc=$?
    echo "v$i [$e] rep $r rc=$rc $(grep -ho '"ms_per_step": [0-9.]*' "$O/v${i}_$r.log")"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
