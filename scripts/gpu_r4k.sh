set -o pipefail
# cached claims open to the block (MM_STEAL, scripts/patches/steal_claims.patch): tail probe, A/B at N=1 and rank 0 of 8
mkdir -p gpurun_out/r4k
MIRROR_MAZE_LIB=exp/tc_steal/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4k/tail_probe_tc_steal.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r4k/tail_probe_tc_steal.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
timeout -k 10 900 python -u scripts/ab.py --tag r4k_ab --config c3:20:3 --config c4:2:2 --config c5s:5:2 --config c2:10:3 --lib exp/base/lib.so --lib exp/steal/lib.so 2>&1 | tail -10 || exit $?
timeout -k 10 600 python -u scripts/ab.py --tag r4k_ab8 --ranks 8 --config c3:20:5 --config c4:4:2 --lib exp/base/lib.so --lib exp/steal/lib.so 2>&1 | tail -6
