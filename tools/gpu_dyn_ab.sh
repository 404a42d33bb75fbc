#!/bin/bash
# Dynamic-tail A/B: kernel times (kbench C2/C3, C5 kernels) and the C2 contract step, default vs AEON_HIP_DYN_TAIL.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; out=gpurun_out/dyn_ab.log; : > $out
V=${DYN:-3}
for rep in 1 2 3; do
  for v in default AEON_HIP_DYN_TAIL=$V; do
    echo -n "$v | " >> $out; timeout -k 10 60 python tools/kbench.py C2 $v 2>&1 | grep "C2 " >> $out || exit 1
  done
done
for v in "" "AEON_HIP_DYN_TAIL=$V"; do
  echo -n "bench [$v] | " >> $out
  env $v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value %.3fM step %.1f us kernel %.1f us' % (d['value']/1e6, d['ms_per_step']*1e3, d['roofline']['kernel_avg_launch_ms']*1e3))" >> $out || exit 1
  echo -n "C5 [$v] | " >> $out
  env $v timeout -k 10 120 python tools/c5_run.py 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('pairs/s %.3fM step %.1f us kernels %.1f us' % (d['value']/1e6, d['ms_per_step']*1e3, d['kernels_ms_per_step']*1e3))" >> $out || exit 1
done
cat $out
