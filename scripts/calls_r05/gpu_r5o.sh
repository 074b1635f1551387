# round 5, call o: per-phase lane utilisation on HEAD's sources (diagnostics build -DMM_LANE_STATS, exp/lanes)
set -o pipefail
mkdir -p gpurun_out/r5o
for C in c3 c5s; do
  MIRROR_MAZE_LIB=exp/lanes/lib.so timeout -k 10 300 python scripts/lane_probe.py --config $C --json gpurun_out/r5o/lane_stats_$C.json > gpurun_out/r5o/lane_stats_$C.txt 2>&1 || exit 1
done
echo r5o done
