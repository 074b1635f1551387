# round 6, call zf: 8 chunks per claim with a longer single-claim zone at the queue's end (MM_CLAIM_TAIL 2 / 4
# x waves x 8 chunks) against HEAD (4 chunks, tail 1), on C3 and on rank 0's share of an 8-way C3 split
set -o pipefail
mkdir -p gpurun_out/r6zf
timeout -k 10 700 python scripts/ab.py --tag r6zf_ab --config c3:20:3 \
  --lib exp/head6/lib.so --lib exp/c8t2/lib.so --lib exp/c8t4/lib.so > gpurun_out/r6zf/ab.txt 2>&1 || { tail -20 gpurun_out/r6zf/ab.txt; exit 1; }
timeout -k 10 700 python scripts/ab.py --tag r6zf_ab8 --config c3:20:3 --ranks 8 \
  --lib exp/head6/lib.so --lib exp/c8t2/lib.so --lib exp/c8t4/lib.so > gpurun_out/r6zf/ab_r8.txt 2>&1 || { tail -20 gpurun_out/r6zf/ab_r8.txt; exit 1; }
tail -4 gpurun_out/r6zf/ab.txt; tail -4 gpurun_out/r6zf/ab_r8.txt
echo r6zf done
