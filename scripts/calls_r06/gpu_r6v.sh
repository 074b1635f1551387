# round 6, call v: is the bare hardware square root / reciprocal already correctly rounded where mm::rsq uses
# its corrected fast form?  (scripts/probe_sqrt_exact.hip, built in the container into scripts/bin/)
set -o pipefail
mkdir -p gpurun_out/r6v
timeout -k 10 120 ./scripts/bin/probe_sqrt_exact > gpurun_out/r6v/probe.txt 2>&1; rc=$?
cat gpurun_out/r6v/probe.txt; exit $rc
