set -o pipefail
# final sources: the -m gpu suite, then the C3 (20-frame launch) and C2 PMC records
mkdir -p gpurun_out/r4p1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4p1/tests.log 2>&1 || { tail -30 gpurun_out/r4p1/tests.log; exit 1; }
tail -3 gpurun_out/r4p1/tests.log
STEPS=20 bash scripts/pmc_bench.sh r4pmc_c3 c3 || exit $?
STEPS=10 bash scripts/pmc_bench.sh r4pmc_c2 c2 || exit $?
echo p1 done
