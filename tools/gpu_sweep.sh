#!/bin/bash
# Kernel tuning sweep: library variants x staging knobs, C2 per-step kernel time (tools/kbench.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/sweep.log; : > $out
for lib in default aeon_amd/variants/*.so; do
  for knobs in default "AEON_HIP_TR=9 AEON_HIP_BANDS=1" "AEON_HIP_TR=16 AEON_HIP_BANDS=1" "AEON_HIP_TR=5 AEON_HIP_BANDS=2" "AEON_HIP_TR=24 AEON_HIP_BANDS=1"; do
    if [ "$lib" = default ]; then L=""; else L="$lib"; fi
    echo -n "$(basename $lib) | " >> $out
    AEON_HIP_LIB="$L" timeout -k 10 120 python tools/kbench.py ${CFG:-C2} $knobs >> $out 2>&1 || { echo "FAILED $lib $knobs" >> $out; exit 1; }
  done
done
cat $out
