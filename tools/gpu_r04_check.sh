#!/bin/bash
# One GPU session: all GPU tests, smoke, the driver's bench line (+ per-launch kernel times of C2/C3
# with tools/kbench.py).  Everything under gpurun_out/.  Usage on the box: bash tools/gpu_r04_check.sh
# PYTEST_ARGS="-k ..." narrows the tests; NO_BENCH=1 stops after smoke.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
python tools/summarize_bench.py gpurun_out/bench.json
for cfg in C2 C3; do timeout -k 10 120 python tools/kbench.py $cfg default 2>&1 | grep -v amdgpu.ids; done
exit 0
