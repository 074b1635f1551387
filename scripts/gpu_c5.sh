#!/bin/bash
# C5 checks: accumulated 4K/64spp/16-bounce frames on the N=64 maze, and the C5 scene at C3 size.
set -o pipefail
OUT=gpurun_out/${1:-c5}; mkdir -p $OUT
timeout -k 10 600 python bench.py --config c5 --accumulate --steps ${C5_STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/c5acc.json 2>$OUT/c5acc.err || { tail $OUT/c5acc.err; exit 1; }
cut -c1-400 $OUT/c5acc.json
timeout -k 10 300 python bench.py --config c5s --steps 5 --no-cpu-baseline > $OUT/c5s.json 2>$OUT/c5s.err || { tail $OUT/c5s.err; exit 1; }
cut -c1-400 $OUT/c5s.json
