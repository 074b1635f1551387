# round 5, call j: A/B of the maze forms' slab specialisation (exp/slab = the working tree) against HEAD
# (exp/glcxp) on C3 / the N=64 scene / C2 / C4; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5j
timeout -k 10 1000 python scripts/ab.py --tag r5j_ab --config c3:20:4 --config c5s:5:2 --config c2:10:2 \
  --config c4:2:1 --lib exp/glcxp/lib.so --lib exp/slab/lib.so \
  > gpurun_out/r5j/ab.txt 2>&1 || { tail -20 gpurun_out/r5j/ab.txt; exit 1; }
tail -10 gpurun_out/r5j/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5j/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5j/tests.log; exit $rc
