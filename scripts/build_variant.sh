#!/bin/bash
# Build the product library from a git revision (or the working tree: "wt")
# into exp/<name>/lib.so, optionally with extra hipcc flags, for A/B runs
# (scripts/ab.py).  Usage: bash scripts/build_variant.sh <name> <rev|wt> [EXTRA flags...]
set -e
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/exp/$NAME
rm -rf $D && mkdir -p $D
if [ "$REV" = wt ]; then
  cp -r $ROOT/include $ROOT/mirror-maze_amd $D/
  rm -rf $D/mirror-maze_amd/build $D/mirror-maze_amd/lib
else
  git -C $ROOT archive $REV include mirror-maze_amd | tar -x -C $D
fi
make -s -j8 -C $D/mirror-maze_amd EXTRA="$*" OUT=$D/lib.so BUILD=$D/build VERIFY=
echo built $D/lib.so
