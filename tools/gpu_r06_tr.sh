#!/bin/bash
# Round 6: C2 rows-per-tile sweep (AEON_HIP_TILE_ROWS) with the C2 parity subset at TR 40.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
AEON_HIP_TILE_ROWS=40 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_parity.py tests/test_pair.py > $OUT/pytest_tr40.log 2>&1
rc=$?; tail -1 $OUT/pytest_tr40.log; [ $rc -eq 0 ] || exit $rc
bash tools/c2_ab.sh base tr24:AEON_HIP_TILE_ROWS=24 tr40:AEON_HIP_TILE_ROWS=40 tr48:AEON_HIP_TILE_ROWS=48 2>&1 | grep -v amdgpu.ids | tee $OUT/c2_ab_tr.txt || exit 1
bash tools/c5_ab.sh base tr40:AEON_HIP_TILE_ROWS=40 tr48:AEON_HIP_TILE_ROWS=48 2>&1 | grep -v amdgpu.ids | tee $OUT/c5_ab_tr.txt
