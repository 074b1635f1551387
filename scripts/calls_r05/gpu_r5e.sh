# round 5, call e: the PMC records of the final sources, second half of scripts/gpu_round.sh pmc; the GPU
# suite (scripts/gpu_round.sh tests); the gather probe
set -o pipefail
export TMPDIR=/tmp
for P in "c5|3|--accumulate" "c5s|5|" "c1|10|" "c4_r8|4|--emulate-ranks 8"; do
  IFS='|' read -r name frames extra <<< "$P"
  STEPS=$frames timeout -k 10 600 bash scripts/pmc_bench.sh pmc_$name ${name%_r8} "$extra" || exit $?
done
mkdir -p gpurun_out/tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/tests/tests.log 2>&1 || { tail -30 gpurun_out/tests/tests.log; exit 1; }
tail -3 gpurun_out/tests/tests.log
timeout -k 10 180 python3 scripts/gather_probe.py > gpurun_out/gather_probe.json 2> gpurun_out/gather_probe.err || { echo "gather probe failed"; exit 1; }
echo r5e done
