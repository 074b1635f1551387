#!/bin/bash
# One-GPU bench lines for the other BASELINE configs (C2, C4) plus the bench-contract test.
set -o pipefail
OUT=gpurun_out/${1:-configs}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "one_json or blocksync or leafinterior" > $OUT/t.log 2>&1; tail -2 $OUT/t.log
for C in c2 c4; do
  timeout -k 10 400 python bench.py --config $C --steps ${STEPS:-5} --no-cpu-baseline > $OUT/$C.json 2>$OUT/$C.err || { tail $OUT/$C.err; exit 1; }
  cut -c1-300 $OUT/$C.json
done
