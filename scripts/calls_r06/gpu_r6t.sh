# round 6, call t: the new long-path tail-ring test and the whole-frame file it sits in
set -o pipefail
mkdir -p gpurun_out/r6t
timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6t/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6t/tests.log; exit $rc
