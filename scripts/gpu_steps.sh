#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit, logging to
# gpurun_out/<tag>/.  A step that ends with an ordinary failure (exit 1, e.g.
# a failed assertion) lets the next step run; a time limit (124/137), an abort
# (134), a segfault (139) or any other code stops the script there -- nothing
# more touches the GPU after a fault.
#   bash scripts/gpu_steps.sh <tag> "<seconds>|<name>|<command>" ...
set -o pipefail
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  secs=${step%%|*}; rest=${step#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "[$(date +%T)] step $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "[$(date +%T)] step $name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: step $name ended with $rc"; exit $rc; fi
done
echo "all steps done"
