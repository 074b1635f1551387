# round 5, call d: the PMC records of the final sources (first half of scripts/gpu_round.sh pmc) and the
# C3 issue-attribution passes (scripts/pmc_issue_record.py sets); record each here afterwards with
# scripts/pmc_record.py / scripts/pmc_issue_record.py
set -o pipefail
export TMPDIR=/tmp
for P in "c3|20|" "c2|10|" "c4|2|" "c3_r8|20|--emulate-ranks 8"; do
  IFS='|' read -r name frames extra <<< "$P"
  STEPS=$frames timeout -k 10 600 bash scripts/pmc_bench.sh pmc_$name ${name%_r8} "$extra" || exit $?
done
SETS=$(python3 -c "import sys; sys.path.insert(0, 'scripts'); import pmc_issue_record as p; print(';'.join(p.ISSUE_SETS))")
STEPS=20 NOSTATS=1 SETS="$SETS" timeout -k 10 600 bash scripts/pmc_bench.sh r5d_issue c3 || exit $?
echo r5d done
