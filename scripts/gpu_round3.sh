# Round-3 GPU record of the current sources: the -m gpu suite, the default bench line, the PMC passes of C3,
# every configuration (scripts/gpu_results.sh) and C5 exactly as BASELINE states it (120 accumulated frames).
set -o pipefail
T=${1:-r3}
bash scripts/gpu_steps.sh $T "900|tests|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "200|bench|python bench.py --steps 20 --warmup 5" || exit $?
bash scripts/pmc_bench.sh ${T}pmc c3 || exit $?
bash scripts/gpu_results.sh ${T}res || exit $?
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 120 --warmup 1 --no-cpu-baseline > gpurun_out/${T}res/c5_acc120.json 2> gpurun_out/${T}res/c5_acc120.err
