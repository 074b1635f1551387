# round 5, call k: rank 0's share of a 2 / 4 / 8-way C3 split on the final sources (scripts/emulated_scaling.sh)
set -o pipefail
bash scripts/gpu_round.sh scaling r5emu || exit $?
echo r5k done
