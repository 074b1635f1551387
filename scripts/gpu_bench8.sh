#!/bin/bash
# bench.py lines for the emulated rank-0 share of an N-way split (N = 1, 2, 4, 8), default options and pixel order.
set -o pipefail
O=gpurun_out/${1:-bench8}; mkdir -p $O
for N in 8 4 2 1; do
  for V in default order0; do
    OPT=""; [ $V = order0 ] && OPT="--opt 17=0"
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --emulate-ranks $N $OPT > $O/n${N}_$V.json 2> $O/n${N}_$V.err || { tail $O/n${N}_$V.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/n${N}_$V.json')); print('N=$N $V', d['ms_per_step'], d['config'].get('frame_contexts'), d['config'].get('frame_contexts_calibration_ms'))"
  done
done
