#!/bin/bash
# Round-3 state of the kernels: decoder GPU tests (parallel window draws), host draw timing, C2
# phase trace, PMC passes + summaries for C2 and C3.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_decoder.py tests/test_integration.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_decoder.log 2>&1 || { tail -30 gpurun_out/pytest_decoder.log; exit 1; }
tail -1 gpurun_out/pytest_decoder.log
timeout -k 10 120 ./tools/make_params_timing > gpurun_out/make_params_timing.txt 2>&1 || exit 1
cat gpurun_out/make_params_timing.txt
timeout -k 10 120 python tools/trace_kernel.py C2 > gpurun_out/trace_c2.log 2>&1 || exit 1
head -12 gpurun_out/trace_c2.log
for cfg in C2 C3; do
  tools/gpu_pmc.sh $cfg > gpurun_out/pmc_$cfg.txt 2>&1 || { echo "pmc $cfg failed"; tail gpurun_out/pmc_$cfg.txt; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc/$cfg $cfg gpurun_out/traffic_r03.json > gpurun_out/pmc_${cfg}_summary.txt || exit 1
  echo "pmc $cfg ok"
done
