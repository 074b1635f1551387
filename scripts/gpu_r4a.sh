set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4a/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4a/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py > gpurun_out/r4a/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r4a/bench.log
timeout -k 10 60 python -u scripts/ring_livelock_repro.py gpurun_out/r4a/repro_r4.json || exit $?
MIRROR_MAZE_LIB=exp/r3lib/libmirror_maze.so timeout -k 10 480 python -u scripts/ring_livelock_repro.py gpurun_out/r4a/repro_r3.json
