#!/bin/bash
# Held-tile form A/B: GPU tests, then C2 kernel / bench lines and the C5 rate for the in-tree library
# (held) and the AEON_HIP_HELD=0 variant.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_lib_ab.sh "$@" || exit 1
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  for i in 1 2; do AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/c5_run.py 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1; done
done
