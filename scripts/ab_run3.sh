set -o pipefail
O=gpurun_out/ab3; mkdir -p $O
for i in 1 2; do
  for c in c3 c5s; do
    MIRROR_MAZE_LIB=exp/cur/lib.so timeout -k 10 200 python scripts/ab_bench.py --config $c --frames 5 --reps 1 default plain 2>&1 | grep -v amdgpu.ids | sed "s/^/$c cur /" >> $O/ab.txt || exit 1
    MIRROR_MAZE_LIB=exp/w768/lib.so timeout -k 10 200 python scripts/ab_bench.py --config $c --frames 5 --reps 1 default plain 2>&1 | grep -v amdgpu.ids | sed "s/^/$c w768 /" >> $O/ab.txt || exit 1
  done
done
