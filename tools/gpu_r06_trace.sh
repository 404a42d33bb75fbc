#!/bin/bash
# Round 6: augment_split timeline (trace build) for C2.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 120 python tools/trace_split.py 2>&1 | grep -v amdgpu.ids | tee $OUT/trace_pipe${1}.txt
