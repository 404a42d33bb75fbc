#!/bin/bash
# The one-launch contrast path (record_kernels.hip): its parity tests and the C3 tests, then C3
# step time with it and without it (AEON_HIP_RECORDS=0), untimed bench runs + per-launch kernel times.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hip_records.py tests/test_hip_parity.py tests/test_decoder.py tests/test_integration.py -m gpu -x -q --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_records.log 2>&1 || { tail -40 gpurun_out/pytest_records.log; exit 1; }
tail -1 gpurun_out/pytest_records.log
for v in 1 0; do
  AEON_HIP_RECORDS=$v timeout -k 10 300 python bench.py --config C3 --steps 30 --warmup 3 --timing-every 0 --no-extra --no-cpu-baseline > gpurun_out/c3_records_$v.json 2>gpurun_out/c3_records_$v.err || { tail -5 gpurun_out/c3_records_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c3_records_$v.json')); print('records=$v', 'C3', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step')"
  AEON_HIP_RECORDS=$v timeout -k 10 120 python tools/kbench.py C3 default 2>&1 | grep -v amdgpu.ids
done
