# round 5, call c: the extended dual-issue microbenchmark, then A/B of the static-LDS grid layout (exp/lay,
# the working tree) against HEAD (exp/base) on C3 / the N=64 scene / C2, then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 120 ./scripts/isa_dual.bin > gpurun_out/r5c/isa_dual.txt 2>&1 || exit $?
timeout -k 10 900 python scripts/ab.py --tag r5c_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 \
  --lib exp/base/lib.so --lib exp/lay/lib.so > gpurun_out/r5c/ab.txt 2>&1 || { tail -20 gpurun_out/r5c/ab.txt; exit 1; }
tail -12 gpurun_out/r5c/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5c/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5c/tests.log; exit $rc
