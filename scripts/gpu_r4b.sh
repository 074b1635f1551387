set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_gpu_errors.py -x -v --timeout 120 --timeout-method thread -k "ring_timeouts or lone_wave" > gpurun_out/r4b/tests.log 2>&1 || { tail -30 gpurun_out/r4b/tests.log; exit 1; }
tail -2 gpurun_out/r4b/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4b/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4b/bench.log | cut -c1-400
timeout -k 10 900 python -u scripts/ab.py --tag r4b --config c3:20:3 --config c5s:5:2 --lib exp/base/lib.so --lib exp/w768/lib.so 2>&1 | tail -8
