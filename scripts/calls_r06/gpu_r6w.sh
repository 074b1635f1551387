# round 6, call w: A/B of HEAD (exp/head3) against 12-byte staged samples (exp/s12 = the working tree: float3
# records instead of float4 slots, global_store_dwordx3 / global_load_dwordx3), then the GPU suite on the tree
set -o pipefail
mkdir -p gpurun_out/r6w
timeout -k 10 600 python scripts/ab.py --tag r6w_ab --config c3:20:3 --config c4:2:2 --config c2:10:2 \
  --lib exp/head3/lib.so --lib exp/s12/lib.so > gpurun_out/r6w/ab.txt 2>&1 || { tail -20 gpurun_out/r6w/ab.txt; exit 1; }
tail -8 gpurun_out/r6w/ab.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > gpurun_out/r6w/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6w/tests.log; exit $rc
