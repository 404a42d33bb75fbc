#!/bin/bash
# One GPU session: parity tests, smoke, the driver's bench command, optional rocprofv3 trace.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>gpurun_out/bench.err && echo "bench ok" \
&& { [ -z "$PROF" ] || { cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 5 --no-cpu-baseline --no-extra > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1 && echo "rocprof ok"; }; }
rc=$?
cd "${GRAFT_REPO_ROOT}"
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log 2>/dev/null; cat gpurun_out/bench.log 2>/dev/null
exit $rc
