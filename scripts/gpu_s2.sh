#!/bin/bash
# Session GPU check: parity tests, smoke, A/B, bench (N=1), rocprof stats.
set -o pipefail
TAG=${1:-s2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== gpu tests"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?; tail -5 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
echo "== ab"; timeout -k 10 600 python scripts/ab_bench.py --frames 5 ${AB:-wp-ldsrec-b1024-w8 default nofuse li-ldsrec} > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }; grep -v amdgpu.ids $OUT/ab.log
[ -z "$AB2" ] || { timeout -k 10 600 python scripts/ab_bench.py --frames 3 --config c5s $AB2 > $OUT/ab2.log 2>&1 || { tail -20 $OUT/ab2.log; exit 1; }; grep -v amdgpu.ids $OUT/ab2.log; }
echo "== bench"; timeout -k 10 600 python bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== rocprof"; cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$OUT/prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT; grep -h "" $OUT/prof/prof_kernel_stats.csv | cut -c1-200; echo done
