# round 6, call y2: C5 as BASELINE.json states it (120 accumulated frames), rocprofv3 --stats of C2 / C4 / C5-120,
# the emulated per-rank scaling (N = 1, 2, 4, 8) and the C3 issue-attribution passes, on HEAD's final sources
set -o pipefail
mkdir -p gpurun_out/r6finres5
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 120 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r6finres5/c5_acc120.json 2> gpurun_out/r6finres5/c5_acc120.err || exit $?
export TMPDIR=/tmp; mkdir -p gpurun_out/r6prof5
for C in "c2|--config c2 --steps 10 --warmup 2" "c4|--config c4 --steps 4 --warmup 1" \
         "c5_acc120|--config c5 --accumulate --steps 120 --warmup 1"; do
  n=${C%%|*}; a=${C#*|}
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r6prof5/$n \
      -o run -- python3 $GRAFT_REPO_ROOT/bench.py $a --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r6prof5/$n.log 2>&1 ) \
    || { echo "rocprof $n failed"; exit 1; }
done
bash scripts/emulated_scaling.sh r6emu5 || exit $?
SETS=$(python3 -c "import sys; sys.path.insert(0, 'scripts'); import pmc_issue_record as p; print(';'.join(p.ISSUE_SETS))")
STEPS=20 NOSTATS=1 SETS="$SETS" timeout -k 10 600 bash scripts/pmc_bench.sh r6y2_issue c3 || exit $?
echo r6y2 done
