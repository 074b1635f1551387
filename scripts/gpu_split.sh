#!/bin/bash
# Tail split: parity tests, A/B at N=1 and the rank-0 share of 8, timeline.
set -o pipefail
O=gpurun_out/${1:-split}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tailsplit or tail_split" --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_bench.py --frames 5 default split default split > $O/ab1.log 2>&1 || { tail $O/ab1.log; exit 1; }; grep -v amdgpu.ids $O/ab1.log
timeout -k 10 300 python scripts/ab_bench.py --frames 10 --ranks 8 default split default split > $O/ab8.log 2>&1 || { tail $O/ab8.log; exit 1; }; grep -v amdgpu.ids $O/ab8.log
timeout -k 10 300 python scripts/ab_bench.py --frames 3 --config c5s default split > $O/ab5.log 2>&1 || { tail $O/ab5.log; exit 1; }; grep -v amdgpu.ids $O/ab5.log
timeout -k 10 300 python scripts/timeline_probe.py --ranks 1,8 --frames 2 --split 1 > $O/tl.log 2>&1 || { tail $O/tl.log; exit 1; }; grep -v amdgpu.ids $O/tl.log
