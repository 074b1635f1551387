# round 6, call zb: the whole-frame GPU tests with the new staged-resolve cases (spp 16 / 24 / 40)
set -o pipefail
mkdir -p gpurun_out/r6zb
timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6zb/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6zb/tests.log; exit $rc
