#!/bin/bash
# C2 contract run at the driver's step count with kernel timing on every k-th step: does timing
# more launches perturb ms_per_step, and how does the sampled kernel average move?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for k in 8 4 2 1 8 1; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extra --timing-every $k 2>/dev/null \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('every', $k, 'ms/step %.4f' % d['ms_per_step'], 'kernel %.2f us' % (r['kernel_avg_launch_ms']*1e3), 'n', r['timed_launches'], 'frac %.3f' % r['frac'])" || exit 1
done
