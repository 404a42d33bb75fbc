#!/bin/bash
# Round 5: the stager (two windows, launch/wait) and the C3 record kernel -- GPU tests + bench line.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_integration.py \
  tests/test_pair.py tests/test_decoder.py tests/test_jpeg.py tests/test_hip_records.py > "$O/pytest_integ.log" 2>&1
AEON_HIP_HOST_PROFILE=0 timeout -k 10 300 python3 -u bench.py > "$O/bench_a.json" 2> "$O/bench_a.err"
echo done
AEON_HIP_HOST_PROFILE=1 timeout -k 10 60 python3 -c "import torch,aeon_amd as A; c=A.Context(0); c.close()" > "$O/vram_flag.txt" 2>&1
