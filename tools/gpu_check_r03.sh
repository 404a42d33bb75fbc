#!/bin/bash
# Round-3 check: all GPU tests, the driver's bench line, per-launch kernel times (tools/kbench.py)
# and a C2 phase trace.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json'))
print('C2', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'us frac', round(d['roofline']['frac'],3))
e=d.get('extra',{})
for k in ('C3','C5','two_streams'):
    if k in e: print(k, round(e[k]['value']), round(e[k]['ms_per_step']*1e3,2), 'us/step')
"
for cfg in C2 C3; do timeout -k 10 120 python tools/kbench.py $cfg default 2>&1 | grep -v amdgpu.ids; done
timeout -k 10 120 python tools/trace_kernel.py C2 > gpurun_out/trace_c2.log 2>&1 && head -6 gpurun_out/trace_c2.log
