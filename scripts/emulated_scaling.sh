#!/bin/bash
# Per-rank cost of an N-way row split of C3 on one GPU (bench.py --emulate-ranks N traces rank 0's rows),
# 20 timed frames as the driver times them, at the default launch size (<= 16 frames) and with all 20 frames
# in one launch (--batch 20).  -> gpurun_out/<tag>/r<N>[_b20].json
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/r1.json 2> $OUT/r1.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --batch 20 > $OUT/r1_b20.json 2> $OUT/r1_b20.err || exit 1
for N in 2 4 8; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --emulate-ranks $N > $OUT/r$N.json 2> $OUT/r$N.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --emulate-ranks $N --batch 20 > $OUT/r${N}_b20.json 2> $OUT/r${N}_b20.err || exit 1
done
echo done
