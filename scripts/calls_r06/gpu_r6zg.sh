# round 6, call zg: repeats on HEAD's final sources for the spread -- the driver's command three times, the rank-0-of-8 emulation
# twice, and the N-GPU path at N = 1 (bench.py --gpus 1 --launcher torchrun: RCCL gather through mm_comm)
set -o pipefail
mkdir -p gpurun_out/r6zg
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6zg/bench_$i.json 2> gpurun_out/r6zg/bench_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --emulate-ranks 8 --no-cpu-baseline > gpurun_out/r6zg/rank0of8_$i.json 2> gpurun_out/r6zg/rank0of8_$i.err || exit 1
done
timeout -k 10 300 python bench.py --gpus 1 --launcher torchrun --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6zg/torchrun_n1.json 2> gpurun_out/r6zg/torchrun_n1.err || exit 1
echo r6zg done
