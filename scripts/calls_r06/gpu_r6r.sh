# round 6, call r: the C5 bench lines again with the corrected C5 PMC record (frames_per_launch 1: C5 accumulates
# one frame per launch) -- 3 frames, and the 120 accumulated frames BASELINE.json states
set -o pipefail
mkdir -p gpurun_out/r6finres3
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 3 --warmup 1 \
  > gpurun_out/r6finres3/c5.json 2> gpurun_out/r6finres3/c5.err || exit $?
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 120 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r6finres3/c5_acc120.json 2> gpurun_out/r6finres3/c5_acc120.err || exit $?
echo r6r done
