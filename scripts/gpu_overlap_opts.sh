#!/bin/bash
# One vs two frame contexts under different kernel options (sharing penalty vs scratch footprint).
set -o pipefail
OUT=gpurun_out/${1:-ovopts}; mkdir -p $OUT
for O in "" ${OPTS:-"--opt 6=3"}; do
 for C in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --contexts $C $O ${EXTRA} > $OUT/b.json 2>$OUT/b.err || { tail $OUT/b.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b.json'));c=d['config'];print('opts [$O] contexts $C', d['ms_per_step'])"
 done
done
