# round 6, call i: A/B against HEAD (exp/head) of a two-trial bank in the rejection sampling (exp/bank2),
# of that + the shading step writing the state unconditionally and the bounce loop rotated to one exit after
# the shading (exp/flow), and of 896-thread blocks at 7 waves per SIMD (exp/w7, HEAD's sources); then the
# grid cell size sweep on HEAD's build (MM_OPT_GRID_CELL: the first cell size tried, percent of the median
# rect extent)
set -o pipefail
mkdir -p gpurun_out/r6i
timeout -k 10 900 python scripts/ab.py --tag r6i_ab --config c3:20:3 --config c5s:5:2 --config c2:10:2 \
  --lib exp/head/lib.so --lib exp/bank2/lib.so --lib exp/flow/lib.so --lib exp/w7/lib.so > gpurun_out/r6i/ab.txt 2>&1 || { tail -20 gpurun_out/r6i/ab.txt; exit 1; }
tail -12 gpurun_out/r6i/ab.txt
timeout -k 10 600 python scripts/ab.py --tag r6i_cell --config c3:20:2 --config c5s:5:1 --lib exp/head/lib.so \
  --variants default cell70 cell80 cell90 cell125 > gpurun_out/r6i/cell.txt 2>&1 || { tail -20 gpurun_out/r6i/cell.txt; exit 1; }
tail -14 gpurun_out/r6i/cell.txt
echo r6i done
