#!/bin/bash
# Repeatability of the headline: the driver's bench command (no extras) several times in one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/rep.log
for i in 1 2 3; do
  for steps in 20 200; do
    timeout -k 10 120 python bench.py --steps $steps --warmup 5 --no-extra --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); r=d['roofline']; print('steps %d value %.0f ms/step %.4f kernel_ms %.4f submit_ms %.4f' % (d['steps'], d['value'], d['ms_per_step'], r['kernel_avg_launch_ms'], d['host_submit_ms_per_step']))" >> gpurun_out/rep.log || exit 1
  done
done
cat gpurun_out/rep.log
