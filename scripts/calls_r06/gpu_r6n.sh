# round 6, call n: PMC records of HEAD's final sources, every configuration -- rocprofv3 --kernel-trace --stats
# + five --pmc passes over bench.py's own launch (scripts/pmc_bench.sh); recorded here with
# scripts/pmc_record.py gpurun_out/pmc_<name> <name> <frames per launch> (c5: 1 -- one launch per accumulated frame)
set -o pipefail
for P in "c3|20|" "c3_r8|20|--emulate-ranks 8" "c3_r4|20|--emulate-ranks 4" "c3_r2|20|--emulate-ranks 2" "c2|10|" \
         "c4|2|" "c4_r8|4|--emulate-ranks 8" "c5|3|--accumulate" "c5s|5|" "c1|10|"; do
  IFS='|' read -r name frames extra <<< "$P"
  STEPS=$frames bash scripts/pmc_bench.sh pmc_$name ${name%_r*} "$extra" || exit $?
done
echo r6n done
