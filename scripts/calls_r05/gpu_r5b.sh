# round 5, call b: the dual-issue microbenchmark (timing + one PMC pass), then the A/B-only placements'
# GPU tests against the -DMM_AB_VARIANTS build (exp/ab/lib.so, scripts/build_variant.sh ab wt -DMM_AB_VARIANTS)
set -o pipefail
mkdir -p gpurun_out/r5b
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/isa_dual.bin > gpurun_out/r5b/isa_dual.txt 2>&1 || exit $?
( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r5b/dual_pmc -o pmc -- $GRAFT_REPO_ROOT/scripts/isa_dual.bin > $GRAFT_REPO_ROOT/gpurun_out/r5b/dual_pmc.log 2>&1 ) || exit $?
MIRROR_MAZE_LIB=$GRAFT_REPO_ROOT/exp/ab/lib.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_random_scene.py -m gpu -v --timeout 300 --timeout-method thread -k "tile_windows_bit_exact or large_scene_bit_exact or small_full_frames_bit_exact or multi_frame_launch_bit_identical" > gpurun_out/r5b/ab_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5b/ab_tests.log; exit $rc
