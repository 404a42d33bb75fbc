#!/bin/bash
# Knob sweep around the current defaults (C2, C3 per-step kernel time).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/sweep4.log; : > $out
for cfg in C2 C3; do
for knobs in default "AEON_HIP_TR=16" "AEON_HIP_TR=24" "AEON_HIP_THREADS=256" "AEON_HIP_THREADS=512" "AEON_HIP_THREADS=256 AEON_HIP_TR=32" "AEON_HIP_STAGE_KB=80 AEON_HIP_TR=48"; do
  timeout -k 10 120 python tools/kbench.py $cfg $knobs 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $knobs" >> $out; exit 1; }
done
done
cat $out
