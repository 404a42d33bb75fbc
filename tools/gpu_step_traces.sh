#!/bin/bash
# rocprofv3 kernel traces of the C5 and C3 steps with the inter-kernel gaps (tools/trace_gaps.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c5" -o run --output-format csv -- python3 "$R/tools/c5_run.py" 30 > "$R/gpurun_out/prof_c5.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_c5.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3" -o run --output-format csv -- python3 "$R/bench.py" --config C3 --steps 30 --warmup 3 --no-extra --no-cpu-baseline > "$R/gpurun_out/prof_c3.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_c3.log"; exit 1; }
cd "$R"
echo "== C5"; python tools/trace_gaps.py gpurun_out/prof_c5 200
echo "== C3"; python tools/trace_gaps.py gpurun_out/prof_c3 200
tail -n 2 gpurun_out/prof_c5.log
