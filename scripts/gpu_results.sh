#!/bin/bash
# bench.py lines (with CPU baselines) for every BASELINE config on one GPU.
set -o pipefail
OUT=gpurun_out/${1:-results}; mkdir -p $OUT
for C in c1 c2 c3 c4 c5s; do
  timeout -k 10 400 python -u bench.py --config $C --steps ${STEPS:-10} --cpu-seconds 8 > $OUT/$C.json 2>$OUT/$C.err || { tail $OUT/$C.err; exit 1; }
  echo "$C done"
done
timeout -k 10 400 python -u bench.py --config c5 --accumulate --steps 3 --warmup 1 --cpu-seconds 8 > $OUT/c5.json 2>$OUT/c5.err || { tail $OUT/c5.err; exit 1; }
echo "c5 done"
