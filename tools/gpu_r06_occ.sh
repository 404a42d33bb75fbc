#!/bin/bash
# Round 6: augment_split with two workgroups per CU (AEON_HIP_SPLIT_OCC=2, RPL=1) -- GPU tests under it, C2 / C5 A/B.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
AEON_HIP_SPLIT_OCC=2 AEON_HIP_SPLIT_RPL=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_occ2.log 2>&1
rc=$?; tail -2 $OUT/pytest_occ2.log; [ $rc -eq 0 ] || exit $rc
bash tools/c2_ab.sh occ2:AEON_HIP_SPLIT_OCC=2,AEON_HIP_SPLIT_RPL=1 occ1:AEON_HIP_SPLIT_OCC=1 tiles:AEON_HIP_SPLIT=0 occ1r1:AEON_HIP_SPLIT_RPL=1 2>&1 | grep -v amdgpu.ids | tee $OUT/c2_ab_occ.txt || exit 1
AEON_HIP_SPLIT_OCC=2 AEON_HIP_SPLIT_RPL=1 AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 120 python tools/trace_split.py 2>&1 | grep -v amdgpu.ids | tee $OUT/trace_occ2.txt || exit 1
bash tools/c5_ab.sh occ2:AEON_HIP_SPLIT_OCC=2,AEON_HIP_SPLIT_RPL=1 tiles:AEON_HIP_SPLIT=0 2>&1 | grep -v amdgpu.ids | tee $OUT/c5_ab_occ.txt
