#!/bin/bash
# Per-rank cost of an N-way row split of C3 on one GPU (bench.py --emulate-ranks N traces rank 0's rows),
# 20 timed frames in one launch as the driver times them (bench.py's default issue mode).
# -> gpurun_out/<tag>/r<N>.json
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/r1.json 2> $OUT/r1.err || exit 1
for N in 2 4 8; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $N > $OUT/r$N.json 2> $OUT/r$N.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $N --opt 21=32 --opt 22=0 > $OUT/r${N}_defer.json 2> $OUT/r${N}_defer.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --emulate-ranks $N --opt 21=0 > $OUT/r${N}_nodefer.json 2> $OUT/r${N}_nodefer.err || exit 1
done
echo done
