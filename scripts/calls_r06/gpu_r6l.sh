# round 6, call l: the GPU suite on the working tree (two-trial bank, unconditional shading state update,
# rotated bounce loop, box check in camera-ray waves only, float n, box address)
set -o pipefail
mkdir -p gpurun_out/r6l
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6l/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6l/tests.log; exit $rc
