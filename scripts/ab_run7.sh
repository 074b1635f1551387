# C3: leaf boxes in LDS (mode 11) vs via L1/L2 (mode 14; A/B build exp/boxg), both with plain and face-range cells
set -o pipefail
O=gpurun_out/ab7; mkdir -p $O
for i in 1 2; do
  for L in base boxg; do
    MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 200 python scripts/ab_bench.py --config c3 --frames 20 --reps 1 default plain 2>&1 | grep -v amdgpu.ids | sed "s/^/c3 $L /" >> $O/ab.txt || exit 1
  done
done
