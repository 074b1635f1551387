# round 6, call x2: final records on HEAD's final sources (12-byte staged samples, per-pixel resolve) -- smoke, the driver's bench
# command, every configuration (scripts/gpu_results.sh), rocprofv3 --kernel-trace --stats of the driver's command
set -o pipefail
bash scripts/gpu_steps.sh r6fin5 \
  "120|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python bench.py --steps 20 --warmup 5" || exit $?
bash scripts/gpu_results.sh r6finres5 || exit $?
bash scripts/prof_bench.sh r6prof5_c3 --steps 20 --warmup 5 || exit $?
echo r6x2 done
