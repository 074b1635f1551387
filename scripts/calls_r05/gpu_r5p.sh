# round 5, call p: bench.py's other issue modes after the fused-RGBA8 change -- float frames, one frame per
# launch (two contexts), and the N-GPU path with float frames at N = 1
set -o pipefail
mkdir -p gpurun_out/r5p
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --frame-format f32 --no-cpu-baseline > gpurun_out/r5p/f32.json 2> gpurun_out/r5p/f32.err || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --batch 1 --no-cpu-baseline > gpurun_out/r5p/batch1.json 2> gpurun_out/r5p/batch1.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --launcher torchrun --steps 10 --warmup 2 --frame-format f32 --no-cpu-baseline > gpurun_out/r5p/torchrun_f32.json 2> gpurun_out/r5p/torchrun_f32.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --launcher torchrun --steps 10 --warmup 2 --batch 1 --no-cpu-baseline > gpurun_out/r5p/torchrun_batch1.json 2> gpurun_out/r5p/torchrun_batch1.err || exit 1
echo r5p done
