#!/bin/bash
# Round 5 (development): resize_generic phase ablation (variants skipping staging / horizontal /
# vertical passes; wrong outputs, timing only) on the C2:CUBIC workload.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for v in base rg1 rg2 rg4 rg7; do export AEON_HIP_SEP_TR=16;
  if [ $v = base ]; then unset AEON_HIP_LIB; else export AEON_HIP_LIB=$R/aeon_amd/variants/$v.so; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/rg_$v" -o run --output-format csv -- python3 "$R/tools/kbench.py" C2:CUBIC default > "$O/rg_$v.log" 2>&1) || exit 1
  python3 - "$O/rg_$v/run_kernel_stats.csv" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "resize_" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], "n=%s avg=%.2f us" % (r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
