#!/bin/bash
# Round 6: PMC passes of the C2 workload with interpolation_method LANCZOS4 / AREA (resize pre-pass kernels).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
for m in LANCZOS4 AREA; do
  tools/gpu_pmc.sh C2:$m > $OUT/pmc_$m.txt 2>&1 || { tail -5 $OUT/pmc_$m.txt; exit 1; }
  python tools/pmc_summary.py "gpurun_out/pmc/C2:$m" "C2:$m" $OUT/traffic_interp.json > $OUT/pmc_${m}_summary.txt || exit 1
done
