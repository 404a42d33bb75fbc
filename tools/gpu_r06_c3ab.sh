#!/bin/bash
# Round 6: C3 record kernel A/B against aeon_amd/variants/prev.so -- record-kernel parity, then the step A/B.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT; T=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_records.py "tests/test_hip_parity.py::test_full_batch_c3_all_records" tests/test_decoder.py > $OUT/pytest_c3_$T.log 2>&1
rc=$?; tail -1 $OUT/pytest_c3_$T.log; [ $rc -eq 0 ] || exit $rc
bash tools/c3_ab.sh new prev:AEON_HIP_LIB=aeon_amd/variants/prev.so 2>&1 | tee $OUT/c3_ab_$T.txt
