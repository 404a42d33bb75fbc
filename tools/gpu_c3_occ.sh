#!/bin/bash
# C3 pass times vs workgroups per CU and rows per tile (kbench, one knob set per line).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "AEON_HIP_WG_PER_CU=3" "AEON_HIP_WG_PER_CU=2" "AEON_HIP_WG_PER_CU=2 AEON_HIP_TR=24" "AEON_HIP_WG_PER_CU=3 AEON_HIP_TR=24" "AEON_HIP_WG_PER_CU=1"; do
  timeout -k 10 120 python tools/kbench.py C3 $v 2>/dev/null | tail -1 || exit 1
done
