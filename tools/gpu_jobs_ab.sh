#!/bin/bash
# Per-step cost A/B: job-table transport (AEON_HIP_JOBS) x kernel-timing sampling (--timing-every).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/jobs_ab.log; : > $out
for m in ${MODES:-0 1 2}; do for te in ${EVERY:-1 4 0}; do
  echo -n "jobs=$m timing_every=$te | " >> $out
  AEON_HIP_JOBS=$m AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-extra --timing-every $te 2>&1 | grep -v amdgpu.ids \
    | python -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('value %.0f ms/step %.4f kernel_ms %.4f frac %.3f submit %.4f' % (d['value'], d['ms_per_step'], r['kernel_avg_launch_ms'], r['frac'], d['host_submit_ms_per_step']))
    else: print(l.strip())" >> $out || { echo FAILED >> $out; exit 1; }
done; done
cat $out
