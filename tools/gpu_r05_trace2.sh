#!/bin/bash
# Round 5: traces of the record kernel variants (one-role 16 phases, 18 phases, split) with SIMD ids.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export AEON_HIP_LIB=aeon_amd/variants/trace.so
AEON_HIP_REC_HELPERS=0 timeout -k 10 120 python3 -u tools/trace_records.py > "$O/trace2_p16.txt" 2>&1
AEON_HIP_REC_HELPERS=0 AEON_HIP_REC_PHASES=18 timeout -k 10 120 python3 -u tools/trace_records.py > "$O/trace2_p18.txt" 2>&1
AEON_HIP_REC_HELPERS=2 timeout -k 10 120 python3 -u tools/trace_records.py > "$O/trace2_split.txt" 2>&1
unset AEON_HIP_LIB
for i in 1 2; do
  for v in "0 0" "0 18" "2 0"; do
    set -- $v
    echo "helpers=$1 phases=$2 $(AEON_HIP_REC_HELPERS=$1 AEON_HIP_REC_PHASES=$2 timeout -k 10 120 python3 tools/kbench.py C3 2>/dev/null | tail -1)" >> "$O/trace2_ab.txt"
  done
done
echo done
