#!/bin/bash
# C5 with the masks on their own stream (as the decoder's post_process runs them) vs one stream:
# decoder GPU tests, then the C5 rate both ways.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decoder.py tests/test_integration.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_decoder.log 2>&1 || { tail -30 gpurun_out/pytest_decoder.log; exit 1; }
tail -1 gpurun_out/pytest_decoder.log
for i in 1 2; do for m in same side; do timeout -k 10 120 python tools/c5_run.py 50 $m 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1; done; done
