# round 5, call m: the fused RGBA8 store (MM_EXT_RGBA8) -- timing against float frames + mm_quantize_rgba8 on
# the driver's launch shape, bit equality; the driver's bench command on it; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5m
timeout -k 10 300 python scripts/rgba8_probe.py --config c3 --frames 20 --reps 3 > gpurun_out/r5m/rgba8_probe.json 2> gpurun_out/r5m/rgba8_probe.err || { tail -5 gpurun_out/r5m/rgba8_probe.err; exit 1; }
tail -1 gpurun_out/r5m/rgba8_probe.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5m/bench.json 2> gpurun_out/r5m/bench.err || { tail -5 gpurun_out/r5m/bench.err; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5m/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5m/tests.log; exit $rc
