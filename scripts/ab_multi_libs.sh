#!/bin/bash
# A/B several builds of the library (MIRROR_MAZE_LIB) on one config, interleaved
# over reps; every line carries the frames' checksum (ck), which must agree
# across builds (bit-identical results).
#   bash scripts/ab_multi_libs.sh <config> <frames> <reps> <lib>...
set -o pipefail
CFG=$1; FR=$2; REPS=$3; shift 3
for i in $(seq 1 $REPS); do
  for L in "$@"; do
    line=$(MIRROR_MAZE_LIB=$L timeout -k 10 200 python scripts/ab_bench.py --config $CFG --frames $FR --reps 1 default 2>&1 \
           | grep -v amdgpu.ids | tail -1) || { echo "failed: $L"; exit 1; }
    echo "$CFG $(basename $(dirname $L)) $line"
  done
done
