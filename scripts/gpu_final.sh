#!/bin/bash
# Final refresh: parity tests, smoke, A/B, bench + rocprof stats, PMC over bench's launch, per-config lines.
set -o pipefail
TAG=${1:-final}
AB="default li-ldsrec" bash scripts/gpu_s2.sh $TAG || exit $?
echo "== pmc (bench launch)"; bash scripts/pmc_bench.sh ${TAG}_pmcb || exit $?
echo "== results"; bash scripts/gpu_results.sh ${TAG}_results || exit $?
echo final done
