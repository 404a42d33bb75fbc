#!/bin/bash
# C2 kernel time vs rows per tile (AEON_HIP_TR): tile counts that quantise evenly onto the
# 768-workgroup persistent grid (TR 25 -> 2304 tiles = 3 per workgroup) against the default 32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for tr in ${TRS:-32 25 28 19 16 38 45}; do
  timeout -k 10 120 python tools/kbench.py C2 AEON_HIP_TR=$tr 2>/dev/null | tail -1 || exit 1
done | tee gpurun_out/tr_sweep.log
