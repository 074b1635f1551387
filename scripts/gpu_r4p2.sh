set -o pipefail
# final sources: the C4, C5 (accumulated) and C5-scene PMC records
STEPS=2 bash scripts/pmc_bench.sh r4pmc_c4 c4 || exit $?
STEPS=3 bash scripts/pmc_bench.sh r4pmc_c5 c5 "--accumulate" || exit $?
STEPS=5 bash scripts/pmc_bench.sh r4pmc_c5s c5s || exit $?
echo p2 done
