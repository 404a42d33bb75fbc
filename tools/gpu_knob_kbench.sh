#!/bin/bash
# Per-launch kernel times (tools/kbench.py) under AEON_HIP_* knob settings, twice each.
# Usage: tools/gpu_knob_kbench.sh CFG "K=V ..." "K=V ..." ...   ("default" = no knob)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cfg=$1; shift
for rep in 1 2; do
  for k in "$@"; do
    timeout -k 10 120 python tools/kbench.py $cfg $k 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
