set -o pipefail
# launch-tail probe with each wave's last new chunk (diagnostics builds): default, young-wave retire, single claims
mkdir -p gpurun_out/r4i
for L in tailclk tc_retire tc_claim1; do
  echo "## $L"
  MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4i/tail_probe_$L.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4i/tail_probe_$L.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
done
