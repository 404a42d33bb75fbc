#!/bin/bash
# C3 step: the 512 KB job table by SDMA + event wait (in-tree) vs the upload kernel (up1m variant):
# untimed C3 bench lines and a rocprof kernel trace of each with the inter-kernel gaps.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  AEON_HIP_LIB="$lib" timeout -k 10 120 python bench.py --config C3 --steps 30 --warmup 3 --timing-every 0 --no-extra --no-cpu-baseline > gpurun_out/c3u.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c3u.json')); print('$v C3', round(d['value']), round(d['ms_per_step']*1e3,1), 'us/step')"
done; done
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  (cd /tmp && AEON_HIP_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_c3u_$v" -o run --output-format csv -- python3 "$R/bench.py" --config C3 --steps 30 --warmup 3 --timing-every 0 --no-extra --no-cpu-baseline > /dev/null 2>&1) || exit 1
  echo "== $v"; python tools/trace_gaps.py gpurun_out/prof_c3u_$v 90 | grep -v "at::native"
done
