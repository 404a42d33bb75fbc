#!/bin/bash
# C2 bench lines (20 steps, no extras) under AEON_HIP_* knob settings, twice each.
# Usage: tools/gpu_knob_bench.sh "K=V ..." "K=V ..." ...   ("default" = no knob)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for k in "$@"; do
    kv=""; [ "$k" != default ] && kv="$k"
    env $kv timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/kb.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/kb.json'))
print('$k', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'submit', round(d['host_submit_ms_per_step']*1e3,2), 'us')"
  done
done
