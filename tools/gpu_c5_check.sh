#!/bin/bash
# GPU tests, then the C5 step: rate (tools/c5_run.py) and a rocprof kernel trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2; do timeout -k 10 120 python tools/c5_run.py 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c5" -o run --output-format csv -- python3 "$R/tools/c5_run.py" 30 > "$R/gpurun_out/prof_c5.log" 2>&1 || exit 1
cd "$R" && python tools/trace_gaps.py gpurun_out/prof_c5 120
