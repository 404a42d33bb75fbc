#!/bin/bash
# Round 5 (development): resize_sep band height sweep on the C2:CUBIC workload.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
for tr in 8 12 16 24; do
  echo "band rows $tr: $(AEON_HIP_SEP_TR=$tr timeout -k 10 200 python3 -u tools/interp_steps.py 30 CUBIC 2>&1 | grep -v amdgpu.ids)"
done
