# round 6, call q: A/B of HEAD (exp/head2) against the working tree (exp/s2: ring_timeout no longer writes two
# constant zero words, whose registers the compiler spilled around every chunk's bounce loop), then the GPU suite
set -o pipefail
mkdir -p gpurun_out/r6q
timeout -k 10 600 python scripts/ab.py --tag r6q_ab --config c3:20:3 --config c5s:5:2 \
  --lib exp/head2/lib.so --lib exp/s2/lib.so > gpurun_out/r6q/ab.txt 2>&1 || { tail -20 gpurun_out/r6q/ab.txt; exit 1; }
tail -5 gpurun_out/r6q/ab.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6q/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6q/tests.log; exit $rc
