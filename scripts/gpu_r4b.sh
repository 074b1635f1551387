set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests/test_gpu_errors.py tests/test_gpu_frames.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "ring or lone_wave or defer or frames" > gpurun_out/r4b/tests.log 2>&1 || { tail -30 gpurun_out/r4b/tests.log; exit 1; }
tail -2 gpurun_out/r4b/tests.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4b/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4b/bench.log | cut -c1-300
timeout -k 10 1000 python -u scripts/ab.py --tag r4b --config c3:20:3 --config c4:2:2 --lib exp/base/lib.so --lib exp/pz/lib.so --lib exp/lds/lib.so --lib exp/w768/lib.so 2>&1 | tail -12
MIRROR_MAZE_LIB=exp/tailclk/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 2 --tail > gpurun_out/r4b/tail_probe.txt 2>&1 || exit $?
cat gpurun_out/r4b/tail_probe.txt | grep -v amdgpu.ids
