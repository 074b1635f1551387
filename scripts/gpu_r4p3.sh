set -o pipefail
# final sources: PMC records of C1 and of rank 0's share of an 8-way C3 / C4 split (bench.py --emulate-ranks 8,
# read back as profiles/pmc_<config>_r8.json), then the emulated scaling table (scripts/emulated_scaling.sh)
STEPS=10 bash scripts/pmc_bench.sh r4pmc_c1 c1 || exit $?
STEPS=20 bash scripts/pmc_bench.sh r4pmc_c3_r8 c3 "--emulate-ranks 8" || exit $?
STEPS=4 bash scripts/pmc_bench.sh r4pmc_c4_r8 c4 "--emulate-ranks 8" || exit $?
bash scripts/emulated_scaling.sh r4emu || exit $?
echo p3 done
