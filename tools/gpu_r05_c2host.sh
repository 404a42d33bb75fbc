#!/bin/bash
# Round 5: C2 host path (compact hot-half tables, one planning pass, LUT memo, own stream) -- parity + timing.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_parity.py \
  tests/test_reference_kats.py tests/test_kats.py > "$O/pytest_c2host.log" 2>&1
AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python3 tools/kbench.py C2 > "$O/c2host_profile.txt" 2>&1
timeout -k 10 300 python3 -u bench.py > "$O/bench_b.json" 2> "$O/bench_b.err"
echo done
