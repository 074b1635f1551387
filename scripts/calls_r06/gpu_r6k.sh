# round 6, call k: A/B of HEAD (exp/head), the two-trial bank with the one-exit bounce loop (exp/flow) and that
# + the grid box check only in waves holding camera rays, n as a float kernel argument, the certificate's box
# address in two adds (exp/s1)
set -o pipefail
mkdir -p gpurun_out/r6k
timeout -k 10 1000 python scripts/ab.py --tag r6k_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 --config c4:2:1 \
  --lib exp/head/lib.so --lib exp/flow/lib.so --lib exp/s1/lib.so > gpurun_out/r6k/ab.txt 2>&1 || { tail -20 gpurun_out/r6k/ab.txt; exit 1; }
tail -14 gpurun_out/r6k/ab.txt
echo r6k done
