#!/bin/bash
# bench.py on every configuration (BASELINE.json configs; C5 as 3 accumulated frames) and rank 0's share of
# an 8-way split of C3 / C4 on one GPU -> gpurun_out/<tag>/<name>.json (scripts/results_table.py).
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -3 $OUT/$name.err; exit 1; }; echo "$name ok"; }
run c1 --config c1
run c2 --config c2
run c3 --config c3 --steps 20 --warmup 5
run c4 --config c4 --steps 4 --warmup 1
run c5s --config c5s
run c5 --config c5 --accumulate --steps 3 --warmup 1
run c3_rank0of8 --config c3 --emulate-ranks 8 --steps 20 --warmup 5 --no-cpu-baseline
run c4_rank0of8 --config c4 --emulate-ranks 8 --steps 4 --warmup 1 --no-cpu-baseline
