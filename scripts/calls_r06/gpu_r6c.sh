# round 6, call c: in-launch chunk resolve (MM_OPT_CHUNK_RESOLVE 1, default) against k_resolve after the launch
# (variant nochunkres) in the working tree's library, C3 / C4 and rank 0 of 8; then the GPU suite
set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 600 python scripts/ab.py --tag r6c_ab --config c3:20:3 --config c4:2:1 \
  --variants default nochunkres > gpurun_out/r6c/ab.txt 2>&1 || { tail -20 gpurun_out/r6c/ab.txt; exit 1; }
timeout -k 10 300 python scripts/ab.py --tag r6c_ab8 --config c3:20:2 --ranks 8 \
  --variants default nochunkres > gpurun_out/r6c/ab8.txt 2>&1 || { tail -20 gpurun_out/r6c/ab8.txt; exit 1; }
tail -6 gpurun_out/r6c/ab.txt; tail -4 gpurun_out/r6c/ab8.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6c/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6c/tests.log; exit $rc
