#!/bin/bash
# A/B two builds of the library (MIRROR_MAZE_LIB) with scripts/ab_bench.py, interleaved.
# usage: bash scripts/ab_libs.sh <tag> <libA> <libB> [variant] [config]
set -o pipefail
TAG=$1; A=$2; B=$3; V=${4:-default}; CFG=${5:-c3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in 1 2; do
  for L in $A $B; do
    echo "## $L"; MIRROR_MAZE_LIB=$L timeout -k 10 200 python scripts/ab_bench.py --config $CFG --frames 5 $V 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done | tee $OUT/ab_libs.log
