# Round-4 PMC records of the final sources, one per configuration, each over bench.py's own launch shape
# (C3: the driver's 20-frame launch), then `python scripts/pmc_record.py gpurun_out/r4pmc_<c> <c> <frames>`
# here: C3 20, C2 10, C4 2, C5 1 (accumulated frames are one launch each), C5s 5.
set -o pipefail
STEPS=20 bash scripts/pmc_bench.sh r4pmc_c3 c3 || exit $?
STEPS=10 bash scripts/pmc_bench.sh r4pmc_c2 c2 || exit $?
STEPS=2 bash scripts/pmc_bench.sh r4pmc_c4 c4 || exit $?
STEPS=3 bash scripts/pmc_bench.sh r4pmc_c5 c5 "--accumulate" || exit $?
STEPS=5 bash scripts/pmc_bench.sh r4pmc_c5s c5s || exit $?
echo all pmc done
