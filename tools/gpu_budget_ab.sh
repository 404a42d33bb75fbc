#!/bin/bash
# Staging-budget variants (fewer rows per tile, more workgroups per CU): launch shape, C2/C5 kernel
# times and bench lines against the in-tree library.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  AEON_HIP_LIB="$lib" AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python tools/kbench.py C2 default 2>&1 | grep "kernel km" | head -2
done
bash tools/gpu_lib_ab.sh "$@"
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/c5_run.py 40 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1
done
