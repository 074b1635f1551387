set -o pipefail
mkdir -p gpurun_out/r4d
for L in tailclk tc_fair tc_retire; do
  echo "## $L"
  MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 2 --tail > gpurun_out/r4d/tail_probe_$L.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4d/tail_probe_$L.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
done
timeout -k 10 900 python -u scripts/ab.py --tag r4d --config c3:20:3 --config c4:2:2 --config c5s:5:2 --lib exp/base/lib.so --lib exp/fair/lib.so --lib exp/retire/lib.so 2>&1 | tail -8
timeout -k 10 600 python -u scripts/ab.py --tag r4d8 --ranks 8 --config c3:20:3 --lib exp/base/lib.so --lib exp/fair/lib.so --lib exp/retire/lib.so 2>&1 | tail -4
