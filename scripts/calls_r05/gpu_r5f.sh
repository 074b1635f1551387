# round 5, call f: the round's final records on the final sources -- smoke, the driver's bench command (plain
# and under rocprofv3 --kernel-trace --stats), every configuration, C5 over 120 accumulated frames, the
# rocprofv3 stats of C2 / C4 / C5-120 (scripts/gpu_round.sh final + scaling)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5fprof
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r5fprof/c3_bench_default -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/r5fprof/c3_bench_default_line.json 2> $GRAFT_REPO_ROOT/gpurun_out/r5fprof/c3_bench_default.err ) || { echo "rocprof bench failed"; exit 1; }
bash scripts/gpu_round.sh final r5f || exit $?
echo r5f done
