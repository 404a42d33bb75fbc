#!/bin/bash
# Round 6: the aeon-surface drop-in -- stager tests, then tools/aeon_path_cpp.cpp (C++, aeon's call sequence).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT; T=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_integration.py tests/test_concurrency.py > $OUT/pytest_stager_$T.log 2>&1
rc=$?; tail -1 $OUT/pytest_stager_$T.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/aeon_path_cpp_$T.txt
for cfg in C2 C1; do for b in pinned pageable; do for m in overlap flush; do
  timeout -k 10 120 ./aeon_amd/aeon_path_cpp $cfg $b $m 24 4 | tee -a $OUT/aeon_path_cpp_$T.txt || exit 1
done; done; done
AEON_HIP_STAGER_SRC_COPY=1 timeout -k 10 120 ./aeon_amd/aeon_path_cpp C2 pinned overlap 24 4 | tee -a $OUT/aeon_path_cpp_$T.txt
