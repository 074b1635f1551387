#!/bin/bash
# rocprofv3 over bench.py's own launches (default issue mode: the timed frames in one multi-frame launch,
# --steps 5 --warmup 0): one --kernel-trace --stats run, then one run per PMC counter set (--pmc never
# combined with other traces), each under its own time limit.  Output: gpurun_out/<tag>/{stats,pmc1..5}.
# Usage: [STEPS=20] [SETS="A B;C D"] [NOSTATS=1] bash scripts/pmc_bench.sh <tag> [config] [extra bench.py args]
# SETS: counter sets separated by ';' (default: the record's five passes); NOSTATS=1 skips the stats run.
# (STEPS: the frames of the run -- bench.py puts up to 32 consecutive frames in one launch, so STEPS=20 profiles
# the driver's own 20-frame C3 launch; default 5)
set -o pipefail
TAG=$1; CFG=${2:-c3}; XARGS=${3:-}; STEPS=${STEPS:-5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="$GRAFT_REPO_ROOT/bench.py --config $CFG --steps $STEPS --warmup 0 --no-cpu-baseline $XARGS"
if [ -z "$NOSTATS" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 $B > $OUT/stats.log 2>&1 \
    || { echo "stats run failed"; tail -5 $OUT/stats.log; exit 1; }
fi
DEFAULT_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES;SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS;GRBM_GUI_ACTIVE GRBM_COUNT"
IFS=';' read -r -a SETLIST <<< "${SETS:-$DEFAULT_SETS}"
i=0
for SET in "${SETLIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $SET -f csv -d $OUT/pmc$i -o pmc -- python3 $B > $OUT/pmc$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
echo pmc done
