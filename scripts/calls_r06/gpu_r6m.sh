# round 6, call m: per-loop lane statistics of HEAD's sources (exp/lanes: -DMM_LANE_STATS) on C3 and the N=64 scene
set -o pipefail
mkdir -p gpurun_out/r6m
MIRROR_MAZE_LIB=exp/lanes/lib.so timeout -k 10 200 python scripts/lane_probe.py --config c3 --json gpurun_out/r6m/lanes_c3.json > gpurun_out/r6m/lanes_c3.txt 2>&1 || exit 1
MIRROR_MAZE_LIB=exp/lanes/lib.so timeout -k 10 200 python scripts/lane_probe.py --config c5s --json gpurun_out/r6m/lanes_c5s.json > gpurun_out/r6m/lanes_c5s.txt 2>&1 || exit 1
cat gpurun_out/r6m/lanes_c3.txt
echo r6m done
