# Tail deferral on / off after round 3's walk changes: C3 (whole frames and rank 0 of 8), C4; PMC of C3 without it
set -o pipefail
O=gpurun_out/ab5; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python scripts/ab_bench.py --config c3 --frames 20 --reps 1 default nodefer 2>&1 | grep -v amdgpu.ids >> $O/c3.txt || exit 1
  timeout -k 10 200 python scripts/ab_bench.py --config c3 --ranks 8 --frames 20 --reps 1 default nodefer 2>&1 | grep -v amdgpu.ids >> $O/c3r8.txt || exit 1
  timeout -k 10 200 python scripts/ab_bench.py --config c4 --frames 2 --reps 1 default nodefer 2>&1 | grep -v amdgpu.ids >> $O/c4.txt || exit 1
done
bash scripts/pmc_bench.sh ab5pmc c3 "--opt 21=0"
