# Round-4 final GPU record of HEAD (after the PMC records are committed; the -m gpu suite ran on the same
# sources in scripts/gpu_r4p1.sh): smoke, the default bench line (the driver's command), every configuration's bench line
# (scripts/gpu_results.sh), C5 as BASELINE states it (120 accumulated frames) and the rocprofv3 --stats
# summaries of the C2 / C4 / C5-120 bench commands.
set -o pipefail
T=${1:-r4f}
bash scripts/gpu_steps.sh $T \
  "120|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python bench.py --steps 20 --warmup 5" || exit $?
bash scripts/gpu_results.sh ${T}res || exit $?
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 120 --warmup 1 --no-cpu-baseline > gpurun_out/${T}res/c5_acc120.json 2> gpurun_out/${T}res/c5_acc120.err || exit $?
export TMPDIR=/tmp; mkdir -p gpurun_out/${T}prof
for C in "c2|--config c2 --steps 10 --warmup 2" "c4|--config c4 --steps 4 --warmup 1" "c5_acc120|--config c5 --accumulate --steps 120 --warmup 1"; do
  n=${C%%|*}; a=${C#*|}
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}prof/$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py $a --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${T}prof/$n.log 2>&1 ) || { echo "rocprof $n failed"; exit 1; }
done
echo final done
