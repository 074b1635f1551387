#!/bin/bash
# bench.py issue-mode calibration check on one GPU: full frame, emulated rank-0 row sets, torchrun gather path.
set -o pipefail
OUT=gpurun_out/${1:-overlap}; mkdir -p $OUT
E_LIST=${E_LIST:-0 2 4 8}
for E in $E_LIST; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --emulate-ranks $E > $OUT/b_e$E.json 2>$OUT/b_e$E.err || { tail $OUT/b_e$E.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b_e$E.json'));c=d['config'];print('emulate $E', d['ms_per_step'], c['frame_contexts'], c['frame_contexts_calibration_ms'])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --no-cpu-baseline > $OUT/tr.json 2>$OUT/tr.err || { tail -30 $OUT/tr.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/tr.json'));c=d['config'];print('torchrun-1', d['ms_per_step'], c['parallelism'], c['frame_contexts'], c['frame_contexts_calibration_ms'])"
