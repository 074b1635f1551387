#!/bin/bash
# One driver for a round's GPU records (replaces round 4's one-off gpu_r4*.sh call scripts and round 3's
# gpu_round3.sh).  Each step puts every GPU command under its own time limit and stops at the first
# failure.  Run it on the box through gpurun, e.g.
#   gpurun -- 'bash scripts/gpu_round.sh tests'
#   gpurun -- 'bash scripts/gpu_round.sh pmc'            # every configuration's PMC passes, then here:
#             python scripts/pmc_record.py gpurun_out/pmc_<name> <name> <frames>   (the list below)
#   gpurun -- 'bash scripts/gpu_round.sh final r4fin2'   # smoke, the driver's bench line, every config,
#                                                         # C5 over 120 frames, rocprofv3 --stats of C2/C4/C5-120
#   gpurun -- 'bash scripts/gpu_round.sh tail exp/a/lib.so exp/b/lib.so'   # launch-tail probe per diagnostics build
#   gpurun -- 'bash scripts/gpu_round.sh scaling r4emu'  # scripts/emulated_scaling.sh
# A/B timing of library builds: scripts/ab.py (builds: scripts/build_variant.sh, patches in scripts/patches/).
set -o pipefail
STEP=$1; shift
case "$STEP" in
  tests)
    mkdir -p gpurun_out/tests
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/tests/tests.log 2>&1 || { tail -30 gpurun_out/tests/tests.log; exit 1; }
    tail -3 gpurun_out/tests/tests.log ;;
  pmc)
    # name | frames per launch (bench.py --steps) | extra bench.py args; record each with
    # `python scripts/pmc_record.py gpurun_out/pmc_<name> <name> <frames>` (C5: 1, one accumulated frame per launch)
    for P in "c3|20|" "c2|10|" "c4|2|" "c5|3|--accumulate" "c5s|5|" "c1|10|" "c3_r8|20|--emulate-ranks 8" \
             "c4_r8|4|--emulate-ranks 8"; do
      IFS='|' read -r name frames extra <<< "$P"
      STEPS=$frames bash scripts/pmc_bench.sh pmc_$name ${name%_r8} "$extra" || exit $?
    done ;;
  final)
    T=${1:-final}
    bash scripts/gpu_steps.sh $T \
      "120|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
      "200|bench|python bench.py --steps 20 --warmup 5" || exit $?
    bash scripts/gpu_results.sh ${T}res || exit $?
    timeout -k 10 300 python bench.py --config c5 --accumulate --steps 120 --warmup 1 --no-cpu-baseline \
      > gpurun_out/${T}res/c5_acc120.json 2> gpurun_out/${T}res/c5_acc120.err || exit $?
    export TMPDIR=/tmp; mkdir -p gpurun_out/${T}prof
    for C in "c2|--config c2 --steps 10 --warmup 2" "c4|--config c4 --steps 4 --warmup 1" \
             "c5_acc120|--config c5 --accumulate --steps 120 --warmup 1"; do
      n=${C%%|*}; a=${C#*|}
      ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}prof/$n \
          -o run -- python3 $GRAFT_REPO_ROOT/bench.py $a --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${T}prof/$n.log 2>&1 ) \
        || { echo "rocprof $n failed"; exit 1; }
    done
    echo final done ;;
  tail)
    mkdir -p gpurun_out/tail
    for L in "$@"; do
      n=$(basename "$(dirname "$L")")
      echo "## $n"
      MIRROR_MAZE_LIB=$L timeout -k 10 300 python -u scripts/timeline_probe.py --config c3 --ranks 1,8 --batch 20 \
        --frames 1 --tail > gpurun_out/tail/tail_probe_$n.txt 2>&1 || exit $?
      grep -v amdgpu.ids gpurun_out/tail/tail_probe_$n.txt | grep -v "XCD [0-7]" | grep -v "block-balanced"
    done ;;
  scaling)
    bash scripts/emulated_scaling.sh ${1:-emu} ;;
  *)
    echo "usage: gpu_round.sh tests | pmc | final [tag] | tail <lib.so>... | scaling [tag]"; exit 2 ;;
esac
