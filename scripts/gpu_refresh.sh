#!/bin/bash
# Full refresh on one GPU: parity tests, smoke, A/B, bench + rocprof stats,
# PMC passes of the default kernel, bench lines for every config.
set -o pipefail
TAG=${1:-refresh}
AB="default li-ldsrec" bash scripts/gpu_s2.sh $TAG || exit $?
echo "== pmc"; bash scripts/pmc.sh ${TAG}_pmc default || exit $?
echo "== results"; bash scripts/gpu_results.sh ${TAG}_results || exit $?
echo refresh done
