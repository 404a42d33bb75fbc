#!/bin/bash
# C2 step time by job-table transport: device planner (default), host planner + upload kernel,
# host planner + zero-copy table (the tile kernel reads the pinned table over PCIe).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; out=gpurun_out/jobs_modes.log; : > $out
b() { echo -n "$* | " >> $out; env "$@" timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-extra --no-cpu-baseline 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.3fM step %.1f us kernel %.1f us submit %.1f us' % (d['value']/1e6, d['ms_per_step']*1e3, d['roofline']['kernel_avg_launch_ms']*1e3, d['host_submit_ms_per_step']*1e3))" >> $out || return 1; }
AEON_HIP_DEVICE_PLAN=0 AEON_HIP_JOBS=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_jobs2.log 2>&1; tail -1 gpurun_out/pytest_jobs2.log >> $out
for rep in 1 2; do
  b AEON_HIP_DEVICE_PLAN=1 && b AEON_HIP_DEVICE_PLAN=0 AEON_HIP_JOBS=3 && b AEON_HIP_DEVICE_PLAN=0 AEON_HIP_JOBS=2 || exit 1
done
cat $out
