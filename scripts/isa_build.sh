#!/bin/bash
# hipcc --save-temps of csrc/trace_kernels.hip with the library's flags into $1 (default /tmp/isa_wt), then the
# census of the default C3 kernel (scripts/isa_census.py --loops).  Usage: bash scripts/isa_build.sh [dir] [EXTRA]
set -e
D=${1:-/tmp/isa_wt}; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $D && cd $D
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -Wall \
  -Wno-unused-function -mllvm -amdgpu-use-amdgpu-trackers=1 -I$ROOT/include -I$ROOT/mirror-maze_amd/csrc "$@" \
  --save-temps -c $ROOT/mirror-maze_amd/csrc/trace_kernels.hip -o $D/tk.o
python3 $ROOT/scripts/isa_census.py $D/trace_kernels-hip-amdgcn-amd-amdhsa-gfx950.s --loops
