# C3 / C5 scene: time vs the CUs the persistent grid covers (MM_OPT_RESERVE_CUS) and vs frames per launch
set -o pipefail
O=gpurun_out/ab8; mkdir -p $O
for c in c3 c5s; do
  timeout -k 10 200 python scripts/ab_bench.py --config $c --frames 10 --reps 1 default reserve64 reserve128 2>&1 | grep -v amdgpu.ids >> $O/cus.txt || exit 1
done
for f in 2 5 10 20 32; do
  timeout -k 10 200 python scripts/ab_bench.py --config c3 --frames $f --reps 1 default 2>&1 | grep -v amdgpu.ids | sed "s/^/frames $f /" >> $O/frames.txt || exit 1
done
