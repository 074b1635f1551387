# round 6, call zd: what the driver runs at round end, on HEAD's final tree -- the GPU suite, smoke, the bench
set -o pipefail
mkdir -p gpurun_out/r6zd
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 450 --timeout-method thread > gpurun_out/r6zd/tests.log 2>&1 || { tail -5 gpurun_out/r6zd/tests.log; exit 1; }
tail -2 gpurun_out/r6zd/tests.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r6zd/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r6zd/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r6zd/bench_noflags.json 2> gpurun_out/r6zd/bench_noflags.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r6zd/bench.json 2> gpurun_out/r6zd/bench.err || exit 1
echo r6zd done
