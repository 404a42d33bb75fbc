#!/bin/bash
# The contract line's kernel timing (one event pair around the timed region's launches) against
# rocprofv3's per-launch average of the same command.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/rb.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/rb.json')); r=d['roofline']
print(round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step kernel', round(r['kernel_avg_launch_ms']*1e3,2), 'frac', round(r['frac'],3), r['timed_launches'], round(r['algorithmic_bytes_per_launch']/1e6,1))"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rb" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-extra --no-cpu-baseline > "$R/gpurun_out/prof_rb.log" 2>&1 || exit 1
cd "$R" && python -c "
import csv,json
for r in csv.DictReader(open('gpurun_out/prof_rb/run_kernel_stats.csv')):
    if 'augment' in r['Name']: print('rocprof', r['Calls'], 'avg', round(float(r['AverageNs'])/1e3,2), 'min', round(float(r['MinNs'])/1e3,2), 'max', round(float(r['MaxNs'])/1e3,2))
l=[x for x in open('gpurun_out/prof_rb.log') if x.startswith('{')][-1]; d=json.loads(l); print('bench under rocprof: kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'step', round(d['ms_per_step']*1e3,2))"
