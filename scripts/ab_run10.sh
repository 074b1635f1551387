# After batching the dequeue: tail deferral on/off, plain cells, 768-thread blocks (exp/cur = working tree, exp/w768)
set -o pipefail
O=gpurun_out/ab10; mkdir -p $O
for i in 1 2; do
  for L in cur w768; do
    MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 200 python scripts/ab_bench.py --config c3 --frames 20 --reps 1 default defer32 plain 2>&1 | grep -v amdgpu.ids | sed "s/^/c3 $L /" >> $O/c3.txt || exit 1
    MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 200 python scripts/ab_bench.py --config c5s --frames 5 --reps 1 default defer32 2>&1 | grep -v amdgpu.ids | sed "s/^/c5s $L /" >> $O/c5s.txt || exit 1
  done
  MIRROR_MAZE_LIB=exp/cur/lib.so timeout -k 10 200 python scripts/ab_bench.py --config c4 --frames 2 --reps 1 default defer32 2>&1 | grep -v amdgpu.ids | sed "s/^/c4 cur /" >> $O/c4.txt || exit 1
  MIRROR_MAZE_LIB=exp/cur/lib.so timeout -k 10 200 python scripts/ab_bench.py --config c3 --ranks 8 --frames 20 --reps 1 default defer32 2>&1 | grep -v amdgpu.ids | sed "s/^/c3r8 cur /" >> $O/c3r8.txt || exit 1
done
