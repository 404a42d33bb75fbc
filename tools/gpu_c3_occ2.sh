#!/bin/bash
# C3 STATS occupancy probe: default library vs the 72-VGPR (7 waves/SIMD) variant at TR 32 / 24 / 20
# (kbench knobs are passed as its arguments: it resets AEON_HIP_TR itself).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; out=gpurun_out/c3_occ2.log; : > $out
run() { echo "== $1 $3" >> $out; env $2 AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python tools/kbench.py C3 $3 2>&1 | grep -v amdgpu.ids | grep "C3 \|km=1" | sort | uniq >> $out || return 1; }
W=AEON_HIP_LIB=aeon_amd/variants/w7.so
run cur "" default && run w7 "$W" AEON_HIP_TR=20 && run w7 "$W" AEON_HIP_TR=16 && run cur "" AEON_HIP_TR=20 && run w7 "$W" AEON_HIP_TR=24 && run cur "" default
cat $out
