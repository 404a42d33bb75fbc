#!/bin/bash
# Knob sweep of the saved previous library (aeon_amd/variants/old.so), C2 per-step kernel time.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/old_sweep.log; : > $out
for knobs in default "AEON_HIP_TR=25 AEON_HIP_STAGE_KB=60" "AEON_HIP_TR=26 AEON_HIP_STAGE_KB=60" "AEON_HIP_TR=38 AEON_HIP_STAGE_KB=60" "AEON_HIP_TR=40 AEON_HIP_STAGE_KB=60" "AEON_HIP_TR=19 AEON_HIP_STAGE_KB=60" "AEON_HIP_TR=32 AEON_HIP_STAGE_KB=60"; do
  echo -n "old | " >> $out
  AEON_HIP_LIB=aeon_amd/variants/old.so timeout -k 10 120 python tools/kbench.py C2 $knobs 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $knobs" >> $out; exit 1; }
done
cat $out
