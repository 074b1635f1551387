# round 6, call j: the GPU suite on the working tree (two-trial bank, unconditional shading state update,
# rotated bounce loop)
set -o pipefail
mkdir -p gpurun_out/r6j
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6j/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6j/tests.log; exit $rc
