#!/bin/bash
# rocprofv3 kernel trace of scripts/ab_bench.py (default variant, 5 frames) for several builds
# (exp/<name>/lib.so) -> gpurun_out/<tag>/<name>/ ; summary with scripts/pmc_kernels.py-style tables.
# usage: bash scripts/prof_libs.sh <tag> <config> <name>...
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for N in "$@"; do
  ( cd /tmp && MIRROR_MAZE_LIB=$GRAFT_REPO_ROOT/exp/$N/lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv \
      -d $OUT/$N -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_bench.py --config $CFG --frames 5 --reps 1 default \
      > $OUT/$N.log 2>&1 ) || { echo "$N failed"; tail -5 $OUT/$N.log; exit 1; }
  echo "$N done"
done
