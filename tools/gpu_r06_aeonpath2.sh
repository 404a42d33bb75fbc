#!/bin/bash
# Round 6: tools/aeon_path_cpp.cpp repeats (variance), C1 and C2, pageable and pinned.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT; T=${1:-x}
: > $OUT/aeon_path_cpp_$T.txt
for rep in 1 2; do for cfg in C1 C2; do for b in pageable pinned; do for m in overlap flush; do
  timeout -k 10 120 ./aeon_amd/aeon_path_cpp $cfg $b $m 24 4 | tee -a $OUT/aeon_path_cpp_$T.txt || exit 1
done; done; done; done
