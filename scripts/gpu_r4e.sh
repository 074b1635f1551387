set -o pipefail
mkdir -p gpurun_out/r4e
MIRROR_MAZE_LIB=exp/tailclk/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4e/tail_probe_kinds.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4e/tail_probe_kinds.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
MIRROR_MAZE_LIB=exp/tailclk/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail --opt 21:0 > gpurun_out/r4e/tail_probe_norings.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4e/tail_probe_norings.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
