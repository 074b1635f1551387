# round 6, call b: A/B of the maze forms' flat walk (exits folded into one end time, face ranges in the high
# half; exp/flat = the working tree) against HEAD (exp/head, banked trials) on C3 / N=64 scene / C2 / C4;
# then the GPU suite on the tree (AB removal, shared-GPU N-rank bench, grid LDS cap test)
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 900 python scripts/ab.py --tag r6b_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 \
  --config c4:2:1 --lib exp/head/lib.so --lib exp/flat/lib.so > gpurun_out/r6b/ab.txt 2>&1 || { tail -20 gpurun_out/r6b/ab.txt; exit 1; }
tail -12 gpurun_out/r6b/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6b/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6b/tests.log; exit $rc
