#!/bin/bash
# Quick GPU iteration: parity tests then the kernel micro-benchmark.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/kbench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kbench.log
