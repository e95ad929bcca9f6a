#!/bin/bash
# Build the library of git revision REV into sudoku_solver_distributed_amd/libsudoku_hip_<TAG>.so
# (A/B against the working tree: SDK_LIB=... or scripts/gpu_ab.sh CFGS="TAG:default cur:default").
#   bash scripts/build_rev.sh HEAD base
set -e
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" sudoku_solver_distributed_amd include | tar -x -C "$TMP"
(cd "$TMP" && python -c "
import sys; sys.path.insert(0, '.')
from sudoku_solver_distributed_amd import build
print(build.build(force=True, out='$ROOT/sudoku_solver_distributed_amd/libsudoku_hip_$TAG.so'))")
rm -rf "$TMP"
