#!/bin/bash
# A/B of one environment knob on the headline: bench.py (C2, no extras) with each value, twice.
# usage: tools/gpu_ab_env.sh VAR "v1 v2 ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
var=$1; vals=$2; shift 2
for rep in 1 2; do
  for v in $vals; do
    env $var=$v timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-extra --no-cpu-baseline "$@" 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); r=d['roofline']; print('$var=$v value %.0f ms/step %.4f kernel_ms %.4f frac %.3f' % (d['value'], d['ms_per_step'], r['kernel_avg_launch_ms'], r['frac']))" || exit 1
  done
done
