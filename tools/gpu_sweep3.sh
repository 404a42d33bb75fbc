#!/bin/bash
# Rows-per-workgroup sweep (prologue amortisation), C2 per-step kernel time.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/sweep3.log; : > $out
for knobs in default "AEON_HIP_TR=24 AEON_HIP_STAGE_KB=40" "AEON_HIP_TR=32 AEON_HIP_STAGE_KB=48" "AEON_HIP_TR=32 AEON_HIP_STAGE_KB=48 AEON_HIP_THREADS=256" "AEON_HIP_TR=40 AEON_HIP_STAGE_KB=64" "AEON_HIP_TR=56 AEON_HIP_STAGE_KB=80" "AEON_HIP_TR=16 AEON_HIP_BANDS=3"; do
  timeout -k 10 120 python tools/kbench.py ${CFG:-C2} $knobs 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $knobs" >> $out; exit 1; }
done
cat $out
