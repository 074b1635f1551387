# round 6, call d: HEAD's sources (banked trials + maze-form walk) -- lane statistics per phase (diagnostics build
# exp/lanes, -DMM_LANE_STATS) on C3 and the N=64 scene, the driver's bench command twice, and the C3 PMC
# passes of the issue / lane-utilisation counters on the driver's 20-frame launch
set -o pipefail
mkdir -p gpurun_out/r6d
MIRROR_MAZE_LIB=exp/lanes/lib.so timeout -k 10 200 python scripts/lane_probe.py --config c3 --json gpurun_out/r6d/lanes_c3.json > gpurun_out/r6d/lanes_c3.txt 2>&1 || exit 1
MIRROR_MAZE_LIB=exp/lanes/lib.so timeout -k 10 200 python scripts/lane_probe.py --config c5s --json gpurun_out/r6d/lanes_c5s.json > gpurun_out/r6d/lanes_c5s.txt 2>&1 || exit 1
cat gpurun_out/r6d/lanes_c3.txt
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6d/bench_$i.json 2> gpurun_out/r6d/bench_$i.err || exit 1
done
python -c "import json;d=json.load(open('gpurun_out/r6d/bench_1.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel_avg_ms'],d['cpu_baseline']['value'])"
STEPS=20 SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES;SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS;GRBM_GUI_ACTIVE GRBM_COUNT" \
  bash scripts/pmc_bench.sh r6d/pmc_c3 c3 || exit 1
echo r6d done
