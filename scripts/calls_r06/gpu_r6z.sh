# round 6, call z: A/B of HEAD (exp/head4) against a per-pixel resolve for spp % 8 == 0 (exp/res8 = the working
# tree: k_resolve8, one thread per pixel, 16-B loads, exact power-of-two mean), then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r6z
timeout -k 10 600 python scripts/ab.py --tag r6z_ab --config c3:20:3 --config c4:2:2 --config c2:10:2 \
  --lib exp/head4/lib.so --lib exp/res8/lib.so > gpurun_out/r6z/ab.txt 2>&1 || { tail -20 gpurun_out/r6z/ab.txt; exit 1; }
tail -8 gpurun_out/r6z/ab.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6z/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6z/tests.log; exit $rc
