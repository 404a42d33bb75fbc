#!/bin/bash
# Staging/workgroup knob sweep for the current library (tools/kbench.py per-step kernel time).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/sweep2.log; : > $out
for cfg in C2 C3; do
  for knobs in default "AEON_HIP_TR=8" "AEON_HIP_TR=24" "AEON_HIP_THREADS=256" "AEON_HIP_THREADS=512" "AEON_HIP_THREADS=256 AEON_HIP_TR=8" "AEON_HIP_BANDS=2"; do
    timeout -k 10 120 python tools/kbench.py $cfg $knobs 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $cfg $knobs" >> $out; exit 1; }
  done
done
cat $out
