#!/bin/bash
# rocprofv3 kernel trace of one bench.py run (args after the tag) -> gpurun_out/<tag>/
# usage: bash scripts/prof_bench.sh <tag> <bench args...>
set -o pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py "$@" \
  > $OUT/bench.json 2> $OUT/bench.err || { echo "failed"; tail -5 $OUT/bench.err; exit 1; }
echo done
