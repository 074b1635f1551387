# round 6, call e: PMC records of the final sources, part 1 -- rocprofv3 --kernel-trace --stats + five --pmc
# passes over bench.py's own launch per configuration (scripts/pmc_bench.sh); recorded here with
# scripts/pmc_record.py gpurun_out/pmc_<name> <name> <frames>
set -o pipefail
for P in "c3|20|" "c3_r8|20|--emulate-ranks 8" "c3_r4|20|--emulate-ranks 4" "c3_r2|20|--emulate-ranks 2" "c2|10|"; do
  IFS='|' read -r name frames extra <<< "$P"
  STEPS=$frames bash scripts/pmc_bench.sh pmc_$name ${name%_r*} "$extra" || exit $?
done
echo r6e done
