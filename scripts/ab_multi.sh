#!/bin/bash
# Time several builds of the library (exp/<name>/lib.so) with scripts/ab_bench.py, interleaved, twice.
# usage: bash scripts/ab_multi.sh <tag> <config> <variant> <name>...
set -o pipefail
TAG=$1; CFG=$2; V=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2; do
  for N in "$@"; do
    echo "## $N"; MIRROR_MAZE_LIB=exp/$N/lib.so timeout -k 10 200 python scripts/ab_bench.py --config $CFG --frames 5 --reps 1 $V 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee $OUT/ab.log
