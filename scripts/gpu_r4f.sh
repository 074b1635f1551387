set -o pipefail
# launch-tail probe: per-SIMD launch order vs chunks and exits (default diagnostics build), and the
# same probe with 512-thread blocks (half the waves per SIMD)
mkdir -p gpurun_out/r4f
MIRROR_MAZE_LIB=exp/tailclk/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4f/tail_probe_simd.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4f/tail_probe_simd.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
MIRROR_MAZE_LIB=exp/occ512/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4f/tail_probe_occ512.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4f/tail_probe_occ512.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
