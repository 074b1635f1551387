# round 6, call o: final records on the final sources -- smoke, the driver's bench command, every configuration
# (scripts/gpu_results.sh), and rocprofv3 --kernel-trace --stats of the driver's exact command
set -o pipefail
bash scripts/gpu_steps.sh r6fin2 \
  "120|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "200|bench|python bench.py --steps 20 --warmup 5" || exit $?
bash scripts/gpu_results.sh r6finres2 || exit $?
bash scripts/prof_bench.sh r6prof2_c3 --steps 20 --warmup 5 || exit $?
echo r6o done
