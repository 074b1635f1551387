set -o pipefail
mkdir -p gpurun_out/r4c
MIRROR_MAZE_LIB=exp/tailclk/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 2 --tail > gpurun_out/r4c/tail_probe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4c/tail_probe.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4c/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4c/tests.log; exit $rc
