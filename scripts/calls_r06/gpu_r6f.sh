# round 6, call f: PMC records of the final sources, part 2 (C4, C4 rank 0 of 8, C5 accumulated, the N=64
# scene at C3 size, C1)
set -o pipefail
for P in "c4|2|" "c4_r8|4|--emulate-ranks 8" "c5|3|--accumulate" "c5s|5|" "c1|10|"; do
  IFS='|' read -r name frames extra <<< "$P"
  STEPS=$frames bash scripts/pmc_bench.sh pmc_$name ${name%_r*} "$extra" || exit $?
done
echo r6f done
