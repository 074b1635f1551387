# round 6, call ze: chunks per queue claim (MM_CLAIM_CHUNKS) re-measured on the final kernel: 4 (HEAD, exp/head6)
# against 8 and 2, on C3 and on rank 0's share of an 8-way C3 split
set -o pipefail
mkdir -p gpurun_out/r6ze
timeout -k 10 700 python scripts/ab.py --tag r6ze_ab --config c3:20:3 \
  --lib exp/head6/lib.so --lib exp/claim8/lib.so --lib exp/claim2/lib.so > gpurun_out/r6ze/ab.txt 2>&1 || { tail -20 gpurun_out/r6ze/ab.txt; exit 1; }
timeout -k 10 700 python scripts/ab.py --tag r6ze_ab8 --config c3:20:3 --ranks 8 \
  --lib exp/head6/lib.so --lib exp/claim8/lib.so --lib exp/claim2/lib.so > gpurun_out/r6ze/ab_r8.txt 2>&1 || { tail -20 gpurun_out/r6ze/ab_r8.txt; exit 1; }
tail -4 gpurun_out/r6ze/ab.txt; tail -4 gpurun_out/r6ze/ab_r8.txt
echo r6ze done
