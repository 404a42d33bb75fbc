#!/bin/bash
# Round 5: C5 A/B -- the gather's two-half LDS-DMA pipeline (default; AEON_HIP_MASK_PIPE=0 = one copy
# phase) and the pair call's gather on a side stream (AEON_HIP_MASK_SIDE=1); mask tests first.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pair.py \
  tests/test_hip_parity.py tests/test_png.py > "$O/pytest_pipe.log" 2>&1
rc=$?; echo "mask tests (pipe) rc=$rc $(tail -n 1 $O/pytest_pipe.log)"; [ $rc -eq 0 ] || exit $rc
export C5_NO_TIMING=1
bash tools/c5_ab.sh pipe nopipe:AEON_HIP_MASK_PIPE=0 side:AEON_HIP_MASK_SIDE=1 sidenopipe:AEON_HIP_MASK_SIDE=1,AEON_HIP_MASK_PIPE=0 > "$O/c5side_ab.txt" 2>&1 || exit $?
cat "$O/c5side_ab.txt"
AEON_HIP_MASK_SIDE=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_pair.py > "$O/pytest_side.log" 2>&1
echo "pair tests (side) rc=$? $(tail -n 1 $O/pytest_side.log)"
