#!/bin/bash
# Round 5: split record kernel with LDS-atomic sums and an overlapped prologue -- parity, A/B, trace.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_records.py \
  "tests/test_hip_parity.py::test_full_batch_c3_all_records" > "$O/pytest_split4.log" 2>&1
for i in 1 2 3; do
  echo "new $(timeout -k 10 120 python3 tools/kbench.py C3 2>/dev/null | tail -1)" >> "$O/split4_ab.txt"
  echo "prev $(AEON_HIP_LIB=aeon_amd/variants/prev.so timeout -k 10 120 python3 tools/kbench.py C3 2>/dev/null | tail -1)" >> "$O/split4_ab.txt"
done
AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 120 python3 -u tools/trace_records.py > "$O/trace5_split.txt" 2>&1
echo done
