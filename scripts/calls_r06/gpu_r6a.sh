# round 6, call a: A/B of banked look-ahead rejection sampling (exp/bank = the working tree) against HEAD
# (exp/base) on C3 / the N=64 scene / C2; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 900 python scripts/ab.py --tag r6a_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 \
  --lib exp/base/lib.so --lib exp/bank/lib.so > gpurun_out/r6a/ab.txt 2>&1 || { tail -20 gpurun_out/r6a/ab.txt; exit 1; }
tail -12 gpurun_out/r6a/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6a/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6a/tests.log; exit $rc
