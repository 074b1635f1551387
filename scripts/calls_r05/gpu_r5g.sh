# round 5, call g: dual-issue forms added to the microbenchmark, then A/B of three kernel edits against HEAD
# (exp/base): the integer-form ray guard (exp/guard), + the rect loop as a do-while (exp/gl), + record address
# by a VGPR shift (exp/gls = the working tree), on C3 / the N=64 scene / C2; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 120 ./scripts/isa_dual.bin > gpurun_out/r5g/isa_dual.txt 2>&1 || exit $?
timeout -k 10 1000 python scripts/ab.py --tag r5g_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 \
  --lib exp/base/lib.so --lib exp/guard/lib.so --lib exp/gl/lib.so --lib exp/gls/lib.so \
  > gpurun_out/r5g/ab.txt 2>&1 || { tail -20 gpurun_out/r5g/ab.txt; exit 1; }
tail -16 gpurun_out/r5g/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5g/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5g/tests.log; exit $rc
