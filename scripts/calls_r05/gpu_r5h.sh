# round 5, call h: A/B of the grid walk edits against HEAD
# (exp/base): integer-form ray guard + the rect loop as a do-while (exp/gl), + the walk's cell as its word's LDS
# address (exp/glc), + compact grids naming rect k as 8 k (exp/glcx = the working tree), on C3 / the N=64 scene /
# C2; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5h

timeout -k 10 1000 python scripts/ab.py --tag r5h_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 \
  --lib exp/base/lib.so --lib exp/gl/lib.so --lib exp/glc/lib.so --lib exp/glcx/lib.so \
  > gpurun_out/r5h/ab.txt 2>&1 || { tail -20 gpurun_out/r5h/ab.txt; exit 1; }
tail -16 gpurun_out/r5h/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5h/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5h/tests.log; exit $rc
