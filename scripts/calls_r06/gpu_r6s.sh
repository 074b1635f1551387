# round 6, call s: the C3 issue-attribution passes on the final sources (scripts/pmc_issue_record.py sets;
# recorded here with scripts/pmc_issue_record.py gpurun_out/r6s_issue c3 20) and a second emulated-scaling run
# (run-to-run spread of rank 0's share)
set -o pipefail
export TMPDIR=/tmp
SETS=$(python3 -c "import sys; sys.path.insert(0, 'scripts'); import pmc_issue_record as p; print(';'.join(p.ISSUE_SETS))")
STEPS=20 NOSTATS=1 SETS="$SETS" timeout -k 10 600 bash scripts/pmc_bench.sh r6s_issue c3 || exit $?
bash scripts/emulated_scaling.sh r6emu3 || exit $?
echo r6s done
