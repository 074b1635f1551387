# A/B of exp/base (HEAD) vs exp/$1 on C3 (20 frames), C4 (2 frames), rank 0 of 8 (20 frames), C5 scene, C2
set -o pipefail
N=$1; O=gpurun_out/ab11_$N; mkdir -p $O
bash scripts/ab_multi_libs.sh c3 20 3 exp/base/lib.so exp/$N/lib.so > $O/c3.txt 2>&1 || exit 1
bash scripts/ab_multi_libs.sh c4 2 2 exp/base/lib.so exp/$N/lib.so > $O/c4.txt 2>&1 || exit 1
bash scripts/ab_multi_libs.sh c5s 5 2 exp/base/lib.so exp/$N/lib.so > $O/c5s.txt 2>&1 || exit 1
bash scripts/ab_multi_libs.sh c2 20 2 exp/base/lib.so exp/$N/lib.so > $O/c2.txt 2>&1 || exit 1
