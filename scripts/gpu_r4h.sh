set -o pipefail
# end-of-queue priority (MM_END_PRIO) and the wider single-claim zone (MM_CLAIM_TAIL=4): tail probe + A/B
mkdir -p gpurun_out/r4h
for L in tc_ep2 tc_ep4t4; do
  echo "## $L"
  MIRROR_MAZE_LIB=exp/$L/lib.so timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 --frames 1 --tail > gpurun_out/r4h/tail_probe_$L.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4h/tail_probe_$L.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
done
timeout -k 10 900 python -u scripts/ab.py --tag r4h --config c3:20:3 --config c4:2:2 --lib exp/base/lib.so --lib exp/ep1/lib.so --lib exp/ep2/lib.so --lib exp/t4/lib.so --lib exp/ep4t4/lib.so 2>&1 | tail -12 || exit $?
timeout -k 10 600 python -u scripts/ab.py --tag r4h8 --ranks 8 --config c3:20:3 --lib exp/base/lib.so --lib exp/ep1/lib.so --lib exp/ep2/lib.so --lib exp/t4/lib.so --lib exp/ep4t4/lib.so 2>&1 | tail -6
