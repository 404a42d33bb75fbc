#!/bin/bash
# Round 6: C2 A/B of store cache policy (AEON_HIP_STORE_AUX) and dynamic-tail rounds (AEON_HIP_TAIL_ROUNDS) variants.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
V=aeon_amd/variants
bash tools/c2_ab.sh base aux0:AEON_HIP_LIB=$V/aux0.so aux3:AEON_HIP_LIB=$V/aux3.so tail1:AEON_HIP_LIB=$V/tail1.so tail3:AEON_HIP_LIB=$V/tail3.so 2>&1 | grep -v amdgpu.ids | tee $OUT/c2_ab_var.txt
