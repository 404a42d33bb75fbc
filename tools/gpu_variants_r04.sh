#!/bin/bash
# Per-launch kernel times (tools/kbench.py) of the in-tree library and of variant builds
# (tools/build_variants.sh, aeon_amd/variants/<name>.so).  Usage: tools/gpu_variants_r04.sh CFG name...
# KBENCH_REAL=1: natural-image sources (tiled img_2112_70) instead of splitmix noise.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
CFG=$1; shift
for rep in 1 2; do
  echo "== in-tree ($rep)"; timeout -k 10 120 python tools/kbench.py $CFG default 2>&1 | grep -v amdgpu.ids || exit 1
  for v in "$@"; do
    echo "== $v ($rep)"; AEON_HIP_LIB="$R/aeon_amd/variants/$v.so" timeout -k 10 120 python tools/kbench.py $CFG default 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo "== real-image sources"; KBENCH_REAL=1 timeout -k 10 120 python tools/kbench.py $CFG default 2>&1 | grep -v amdgpu.ids
