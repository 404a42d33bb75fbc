#!/bin/bash
# Round profile set: GPU parity tests, smoke, the driver's bench command, then rocprofv3 kernel
# stats of the C2 contract run (100 steps) and of the C3 kernels (tools/kbench.py C3).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
echo "bench ok"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --no-extra > "$R/gpurun_out/prof_c2.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_c2.log"; exit 1; }
echo "rocprof C2 ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c3" -o run --output-format csv -- python3 "$R/tools/kbench.py" C3 default > "$R/gpurun_out/prof_c3.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_c3.log"; exit 1; }
echo "rocprof C3 ok"
