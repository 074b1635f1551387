set -o pipefail
# launch-tail probe with each wave's last new chunk (diagnostics builds): default, the end-of-queue split
# (MM_END_SPLIT=16), young-wave retire, single claims; then the A/B of the split (N=1 and rank 0 of 8)
mkdir -p gpurun_out/r4i
for L in tailclk tc_es16 tc_retire tc_claim1; do
  echo "## $L"
  MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4i/tail_probe_$L.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4i/tail_probe_$L.txt | grep -v "XCD [0-7]" | grep -v "block-balanced" | grep -v "launch order [0-9]:"
done
timeout -k 10 900 python -u scripts/ab.py --tag r4i_ab --config c3:20:3 --config c4:2:2 --lib exp/base/lib.so --lib exp/es16/lib.so --lib exp/es32/lib.so 2>&1 | tail -8 || exit $?
timeout -k 10 600 python -u scripts/ab.py --tag r4i_ab8 --ranks 8 --config c3:20:3 --lib exp/base/lib.so --lib exp/es16/lib.so --lib exp/es32/lib.so 2>&1 | tail -4
