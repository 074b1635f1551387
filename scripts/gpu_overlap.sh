set -o pipefail
OUT=gpurun_out/${1:-overlap}; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 10 --no-cpu-baseline > $OUT/b1.json 2>$OUT/b1.err || { tail $OUT/b1.err; exit 1; }; cut -c1-200 $OUT/b1.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --contexts 2 --no-cpu-baseline > $OUT/tr2.json 2>$OUT/tr2.err || { tail -30 $OUT/tr2.err; exit 1; }; cut -c1-200 $OUT/tr2.json
timeout -k 10 300 python scripts/scaling_probe.py --frames 10 --overlap own > $OUT/probe.log 2>&1; grep N= $OUT/probe.log
timeout -k 10 300 python scripts/scaling_probe.py --frames 10 --overlap own --gate 0 > $OUT/probe0.log 2>&1; grep N= $OUT/probe0.log
timeout -k 10 300 python scripts/scaling_probe.py --frames 10 > $OUT/probe_seq.log 2>&1; grep N= $OUT/probe_seq.log
