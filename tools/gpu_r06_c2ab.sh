#!/bin/bash
# Round 6: C2 / C5 A/B of the current library against aeon_amd/variants/prev.so, with the C2 / C5 parity subset.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT; T=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_parity.py tests/test_pair.py > $OUT/pytest_c2_$T.log 2>&1
rc=$?; tail -1 $OUT/pytest_c2_$T.log; [ $rc -eq 0 ] || exit $rc
bash tools/c2_ab.sh new prev:AEON_HIP_LIB=aeon_amd/variants/prev.so 2>&1 | grep -v amdgpu.ids | tee $OUT/c2_ab_$T.txt || exit 1
bash tools/c5_ab.sh new prev:AEON_HIP_LIB=aeon_amd/variants/prev.so 2>&1 | grep -v amdgpu.ids | tee $OUT/c5_ab_$T.txt
