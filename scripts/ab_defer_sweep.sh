#!/bin/bash
# MM_OPT_DEFER sweep (runtime option, one build) on C3, C4, the C5 scene and rank 0 of an 8-way C3 split.
# usage: bash scripts/ab_defer_sweep.sh <tag>
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
V="default defer40 defer48 defer56"
for C in c3 c4 c5s; do
  timeout -k 10 300 python scripts/ab_bench.py --config $C --reps 3 $V 2>&1 | grep -v amdgpu.ids > $OUT/$C.log || exit 1
done
timeout -k 10 300 python scripts/ab_bench.py --config c3 --ranks 8 --frames 10 --reps 3 $V 2>&1 | grep -v amdgpu.ids > $OUT/c3_rank0of8.log || exit 1
echo sweep done
