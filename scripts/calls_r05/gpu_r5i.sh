# round 5, call i: A/B of staged cell words holding their lists' LDS byte addresses (exp/glcxp = the working
# tree) against HEAD (exp/glcx) on C3 / the N=64 scene / C2 / C4; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5i
timeout -k 10 1000 python scripts/ab.py --tag r5i_ab --config c3:20:4 --config c5s:5:2 --config c2:10:2 \
  --config c4:2:1 --lib exp/glcx/lib.so --lib exp/glcxp/lib.so \
  > gpurun_out/r5i/ab.txt 2>&1 || { tail -20 gpurun_out/r5i/ab.txt; exit 1; }
tail -10 gpurun_out/r5i/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5i/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5i/tests.log; exit $rc
