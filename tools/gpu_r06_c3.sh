#!/bin/bash
# Round 6: C3 record-kernel shapes -- parity under 17 row phases + 1 helper, then the step A/B.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
AEON_HIP_REC_PHASES=17 AEON_HIP_REC_HELPERS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_records.py "tests/test_hip_parity.py::test_full_batch_c3_all_records" > $OUT/pytest_c3_17.log 2>&1
rc=$?; tail -1 $OUT/pytest_c3_17.log; [ $rc -eq 0 ] || exit $rc
bash tools/c3_ab.sh base p17h1:AEON_HIP_REC_PHASES=17,AEON_HIP_REC_HELPERS=1 p16h1:AEON_HIP_REC_HELPERS=1 2>&1 | tee $OUT/c3_ab_phases.txt
