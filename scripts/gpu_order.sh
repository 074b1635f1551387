set -o pipefail
O=gpurun_out/order; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "order" --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/ab_bench.py --frames 5 default order1 default order1 > $O/ab1.log 2>&1 || { tail $O/ab1.log; exit 1; }; grep -v amdgpu.ids $O/ab1.log
timeout -k 10 300 python scripts/ab_bench.py --frames 10 --ranks 8 default order1 default order1 > $O/ab8.log 2>&1 || { tail $O/ab8.log; exit 1; }; grep -v amdgpu.ids $O/ab8.log
timeout -k 10 300 python scripts/ab_bench.py --frames 3 --config c5s default order1 > $O/ab5.log 2>&1 || { tail $O/ab5.log; exit 1; }; grep -v amdgpu.ids $O/ab5.log
timeout -k 10 300 python scripts/timeline_probe.py --ranks 1,8 --frames 2 --order 1 > $O/tl1.log 2>&1 || { tail $O/tl1.log; exit 1; }; grep -v amdgpu.ids $O/tl1.log
timeout -k 10 300 python scripts/timeline_probe.py --ranks 1,8 --frames 2 --order 0 > $O/tl0.log 2>&1 || { tail $O/tl0.log; exit 1; }; grep -v amdgpu.ids $O/tl0.log
