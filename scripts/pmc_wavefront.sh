#!/bin/bash
# rocprofv3 summary + PMC passes of MM_PIPE_WAVEFRONT on C3.  Run at commit 04a553c (before its retirement) it
# profiled the round-1 flattened pipeline (trace_wave.hip: k_wf_generate/extend/shade), the evidence for
# retiring it (profiles/r02/wavefront_pmc.txt); MM_PIPE_WAVEFRONT now runs the wave-persistent
# kernel with the mirror-tail queue.  One run per counter set, each under its own time limit.
# Usage: bash scripts/pmc_wavefront.sh <tag>
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="$GRAFT_REPO_ROOT/scripts/ab_bench.py --reps 1 --frames 2 wave"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/stats -o run -- python3 $B > $OUT/stats.log 2>&1 \
  || { echo "stats run failed"; tail -5 $OUT/stats.log; exit 1; }
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $SET -f csv -d $OUT/pmc$i -o pmc -- python3 $B > $OUT/pmc$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
echo pmc done
