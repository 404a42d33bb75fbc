#!/bin/bash
# C2 bench line at K = 20 (the driver's) and K = 100 / 400 steps: the fixed cost of one timed region
# (first call's host planning on an idle GPU, first dispatch, closing synchronize) over K.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for k in 20 100 400; do
    timeout -k 10 120 python bench.py --steps $k --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/steps.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/steps.json'))
print('K=$k', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step; launch span', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'us')"
  done
done
