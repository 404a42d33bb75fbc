#!/bin/bash
# Round 6: augment_split with three staging buffers -- GPU tests, C2 A/B against augment_tiles, a trace.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu3.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu3.log; [ $rc -eq 0 ] || exit $rc
bash tools/c2_ab.sh split:AEON_HIP_SPLIT=1 tiles:AEON_HIP_SPLIT=0 2>&1 | grep -v amdgpu.ids | tee $OUT/c2_pipe_ab.txt
AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 120 python tools/trace_split.py 2>&1 | grep -v amdgpu.ids | tee $OUT/trace_pipe.txt
bash tools/c5_ab.sh split:AEON_HIP_SPLIT=1 tiles:AEON_HIP_SPLIT=0 2>&1 | grep -v amdgpu.ids | tee $OUT/c5_pipe_ab.txt
