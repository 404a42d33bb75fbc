#!/bin/bash
# augment_rows (streaming, no LDS staging) vs the tile kernel on C2: parity of the direct-call
# tests, per-launch kernel times over TR, the C2 bench line, and rocprof stats of it.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py -m gpu -q -x --timeout 120 --timeout-method thread \
  -k "full_batch_c2 or full_batch_c5 or golden or configs_fixed or edge_cases or zero_copy or direct" > gpurun_out/rows_pytest.log 2>&1 || { tail -30 gpurun_out/rows_pytest.log; exit 1; }
tail -1 gpurun_out/rows_pytest.log
for rep in 1 2; do
  for tr in 0 28 16 56 ${EXTRA_TR:-}; do
    echo -n "TR=$tr | "; timeout -k 10 120 python tools/kbench.py C2 AEON_HIP_ROWS_TR=$tr 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/rows_bench.json 2>gpurun_out/rows_bench.err || { tail -5 gpurun_out/rows_bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/rows_bench.json'))
print('C2', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'us frac', round(d['roofline']['frac'],3))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rows" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --no-extra > "$R/gpurun_out/prof_rows.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_rows.log"; exit 1; }
grep -E "augment" "$R/gpurun_out/prof_rows/run_kernel_stats.csv" | cut -d, -f1-4
