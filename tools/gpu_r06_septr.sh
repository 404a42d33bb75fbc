#!/bin/bash
# Round 6: resize_sep band height (AEON_HIP_SEP_TR) A/B on the C2 workload per interpolation method.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
for round in 1 2; do
  for tr in 16 8 32; do
    echo "== SEP_TR $tr" | tee -a $OUT/interp_septr.txt
    AEON_HIP_SEP_TR=$tr timeout -k 10 200 python tools/interp_steps.py 20 CUBIC,AREA,LANCZOS4 2>&1 | grep -v amdgpu.ids | tee -a $OUT/interp_septr.txt || exit 1
  done
done
