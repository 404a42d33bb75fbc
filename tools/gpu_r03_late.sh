#!/bin/bash
# Late round-3 checks: all GPU tests, C5 with the masks on a side stream vs one stream, and C3
# kernel times with the 9-dot4 pass-1 sums against the sums12 variant (the 12-dot4 form).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2; do for m in same side; do timeout -k 10 120 python tools/c5_run.py 50 $m 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1; done; done
for i in 1 2 3; do for v in cur sums12; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  echo -n "$v | "; AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/kbench.py C3 default 2>&1 | grep -v amdgpu.ids || exit 1
done; done
