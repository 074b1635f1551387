# A/B of two library builds (exp/base = HEAD, exp/<name> = working tree) on C3 (20 frames) and the C5 scene
set -o pipefail
N=${1:-slab}; O=gpurun_out/ab6_$N; mkdir -p $O
bash scripts/ab_multi_libs.sh c3 20 3 exp/base/lib.so exp/$N/lib.so > $O/c3.txt 2>&1 || exit 1
bash scripts/ab_multi_libs.sh c5s 5 2 exp/base/lib.so exp/$N/lib.so > $O/c5s.txt 2>&1 || exit 1
