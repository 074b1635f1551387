# round 6, call za: A/B of HEAD (exp/head4) against a per-pixel resolve for spp % 8 == 0 (exp/res8 = the working
# tree: k_resolve8, one thread per pixel, 16-B loads; the mean as an exact power-of-two multiply in every resolve), then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r6za
timeout -k 10 600 python scripts/ab.py --tag r6za_ab --config c3:20:3 --config c4:2:2 --config c2:10:3 --config c5s:5:2 \
  --lib exp/head4/lib.so --lib exp/res8/lib.so > gpurun_out/r6za/ab.txt 2>&1 || { tail -20 gpurun_out/r6za/ab.txt; exit 1; }
tail -8 gpurun_out/r6za/ab.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6za/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6za/tests.log; exit $rc
