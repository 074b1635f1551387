#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprofv3 kernel stats.
# Usage (from repo root on the box): bash scripts/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== env" ; (nproc; rocm-smi --showproductname 2>/dev/null | head -20) > $OUT/env.txt 2>&1
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1 || { echo build failed; tail -20 $OUT/build.log; exit 1; }
[ -n "$SKIP_TESTS" ] || { echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/gpu_tests.log 2>&1; rc=$?; tail -15 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc; }
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
echo "== ab"; timeout -k 10 600 python scripts/ab_bench.py --config ${AB_CONFIG:-c3} ${AB:-wp-ldsrec-b1024-w8 mega-lds-b512} > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }; cat $OUT/ab.log
[ -z "$AB_ONLY" ] || exit 0
echo "== bench"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "== rocprof"; cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$OUT/prof -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT; find $OUT/prof -name "*stats*" | head; echo done
