#!/bin/bash
# Multi-frame launches: parity tests, then bench.py at the rank-0 share of N = 8, 4, 2, 1 (calibrated issue mode).
set -o pipefail
O=gpurun_out/${1:-batch}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "multi_frame or bench_prints" --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for N in 8 4 2 1; do
  timeout -k 10 300 python -u bench.py --steps 16 --warmup 2 --no-cpu-baseline --emulate-ranks $N > $O/n$N.json 2> $O/n$N.err || { tail $O/n$N.err; exit 1; }
  python -c "import json; d=json.load(open('$O/n$N.json')); c=d['config']; print('N=$N', d['ms_per_step'], 'ms/frame', d['value'], c['frame_contexts'], c['frames_per_launch'], c['frame_contexts_calibration_ms'])"
done
