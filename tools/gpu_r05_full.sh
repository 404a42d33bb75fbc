#!/bin/bash
# Round 5: the whole GPU test suite, then the decoder reproducer combination twice more.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > "$O/pytest_full.log" 2>&1
echo "full rc=$? $(tail -n 1 $O/pytest_full.log)"
for i in 1 2; do
  timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
    "tests/test_integration.py::test_provider_base_post_process_drop_in" "tests/test_integration.py::test_stager_errors" \
    tests/test_jpeg.py tests/test_decoder.py > "$O/repro_$i.log" 2>&1
  rc=$?
  echo "repro$i rc=$rc $(tail -n 1 $O/repro_$i.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
