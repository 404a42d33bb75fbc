#!/bin/bash
# Round 5: concurrency + integration + JPEG tests (512-lane Huffman default), then the bench line.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_concurrency.py > "$O/pytest_conc2.log" 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_integration.py tests/test_jpeg.py tests/test_decoder.py > "$O/pytest_b.log" 2>&1
timeout -k 10 600 python3 -u bench.py > "$O/bench_c.json" 2> "$O/bench_c.err"
echo done
