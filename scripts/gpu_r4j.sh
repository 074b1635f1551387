set -o pipefail
# speed-sized claims (MM_SPEED_CLAIMS, scripts/patches/speed_claims.patch): tail probe, then A/B at N=1 and rank 0 of 8
mkdir -p gpurun_out/r4j
for L in tc_sc4; do
  echo "## $L"
  MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4j/tail_probe_$L.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4j/tail_probe_$L.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
done
timeout -k 10 900 python -u scripts/ab.py --tag r4j_ab --config c3:20:3 --config c4:2:2 --config c5s:5:2 --lib exp/base/lib.so --lib exp/sc4/lib.so --lib exp/sc8/lib.so 2>&1 | tail -10 || exit $?
timeout -k 10 600 python -u scripts/ab.py --tag r4j_ab8 --ranks 8 --config c3:20:4 --lib exp/base/lib.so --lib exp/sc4/lib.so --lib exp/sc8/lib.so 2>&1 | tail -4
