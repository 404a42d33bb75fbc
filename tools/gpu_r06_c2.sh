#!/bin/bash
# Round 6: C2 A/B (augment_split vs augment_tiles) + split trace, no tests.  $1: tag.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT; T=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_parity.py -k "c2 or golden" > $OUT/pytest_$T.log 2>&1
rc=$?; tail -1 $OUT/pytest_$T.log; [ $rc -eq 0 ] || exit $rc
bash tools/c2_ab.sh split:AEON_HIP_SPLIT=1 tiles:AEON_HIP_SPLIT=0 ${2} 2>&1 | grep -v amdgpu.ids | tee $OUT/c2_ab_$T.txt || exit 1
AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 120 python tools/trace_split.py 2>&1 | grep -v amdgpu.ids | tee $OUT/trace_$T.txt
