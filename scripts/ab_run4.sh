# Deferral A/B on C3 and on the N=64 scene (mode 14 now holds its records in LDS): ab_bench, then bench.py on
# C5 (3 accumulated frames) with and without deferral, then the PMC passes of the C5 scene at C3 size.
set -o pipefail
O=gpurun_out/ab4; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python scripts/ab_bench.py --config c5s --frames 5 --reps 1 default defer32 defer16 2>&1 | grep -v amdgpu.ids >> $O/c5s.txt || exit 1
  timeout -k 10 200 python scripts/ab_bench.py --config c3 --frames 10 --reps 1 default nodefer defer16 2>&1 | grep -v amdgpu.ids >> $O/c3.txt || exit 1
done
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 3 --warmup 1 --no-cpu-baseline > $O/c5_default.json 2> $O/c5_default.err || exit 1
timeout -k 10 300 python bench.py --config c5 --accumulate --steps 3 --warmup 1 --no-cpu-baseline --opt 21=32 > $O/c5_defer32.json 2> $O/c5_defer32.err || exit 1
bash scripts/pmc_bench.sh ab4pmc c5s
