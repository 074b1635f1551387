# round 6, call zc: A/B of HEAD (exp/head5, the two-trial bank) against a three-trial bank (exp/bank3 = the
# working tree; a parked path keeps two), then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r6zc
timeout -k 10 700 python scripts/ab.py --tag r6zc_ab --config c3:20:4 --config c5s:5:2 --config c2:10:2 \
  --lib exp/head5/lib.so --lib exp/bank3/lib.so > gpurun_out/r6zc/ab.txt 2>&1 || { tail -20 gpurun_out/r6zc/ab.txt; exit 1; }
tail -8 gpurun_out/r6zc/ab.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6zc/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6zc/tests.log; exit $rc
