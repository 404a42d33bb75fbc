#!/bin/bash
# Event fences A/B: the in-tree library (timing + ring events without system-scope fences) and the
# AEON_HIP_DONE_FENCE=1 variant: C2 bench lines, and a rocprof kernel trace of 100 steps with the
# inter-kernel gaps (tools/trace_gaps.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
summ() { python -c "
import json,sys; d=json.load(open('$1'))
print('$2', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'submit', round(d['host_submit_ms_per_step']*1e3,2), 'us')"; }
for rep in 1 2; do
  for v in cur "$@"; do
    lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
    AEON_HIP_LIB="$lib" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/ev_$v.json 2>/dev/null || exit 1
    summ gpurun_out/ev_$v.json "$v 20 steps"
  done
done
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  (cd /tmp && AEON_HIP_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ev_$v" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --no-extra > "$R/gpurun_out/prof_ev_$v.log" 2>&1) || exit 1
  echo "== $v"; python tools/trace_gaps.py gpurun_out/prof_ev_$v 100
done
