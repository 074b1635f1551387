# Dequeue claim size A/B (exp/claim<k>: -DMM_CLAIM_CHUNKS=k; claim1 = one chunk per atomicAdd as before)
set -o pipefail
O=gpurun_out/ab9; mkdir -p $O
L="exp/claim1/lib.so exp/claim2/lib.so exp/claim4/lib.so exp/claim8/lib.so"
bash scripts/ab_multi_libs.sh c3 20 2 $L > $O/c3.txt 2>&1 || exit 1
bash scripts/ab_multi_libs.sh c5s 5 2 $L > $O/c5s.txt 2>&1 || exit 1
bash scripts/ab_multi_libs.sh c2 20 2 $L > $O/c2.txt 2>&1 || exit 1
