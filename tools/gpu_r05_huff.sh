#!/bin/bash
# Round 5: jpeg_huff at 512 lanes (two files per CU) against 1,024 -- parity and kernel time per window.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
AEON_HIP_JPEG_HUFF_LANES=512 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_jpeg.py > "$O/pytest_huff512b.log" 2>&1
for l in 1024 512; do
  echo "== lanes $l" >> "$O/huff_lanes2.txt"
  JPEG_PROBE_GPU_ONLY=1 AEON_HIP_JPEG_HUFF_LANES=$l timeout -k 10 300 python3 -u tools/jpeg_probe.py 256 512 1024 2>/dev/null | grep "^gpu" >> "$O/huff_lanes2.txt"
done
echo done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_jpeg.py tests/test_decoder.py > "$O/pytest_huff1024b.log" 2>&1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_concurrency.py tests/test_integration.py > "$O/pytest_conc.log" 2>&1
timeout -k 10 600 python3 -u bench.py > "$O/bench_c.json" 2> "$O/bench_c.err"
echo done2
