# round 5, call l: A/B of kernel-argument reloads instead of spilled masks (exp/rl = the working tree) against HEAD
# (exp/glcxp) on C3 / the N=64 scene / C2 / C4; then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r5l
timeout -k 10 1000 python scripts/ab.py --tag r5l_ab --config c3:20:4 --config c5s:5:2 --config c2:10:2 \
  --config c4:2:1 --lib exp/glcxp/lib.so --lib exp/rl/lib.so \
  > gpurun_out/r5l/ab.txt 2>&1 || { tail -20 gpurun_out/r5l/ab.txt; exit 1; }
tail -10 gpurun_out/r5l/ab.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5l/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5l/tests.log; exit $rc
