#!/bin/bash
# Round 6: C3 record kernel with the helpers' job fields in SGPRs -- parity (16+2 and 17+1), step A/B.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_records.py "tests/test_hip_parity.py::test_full_batch_c3_all_records" > $OUT/pytest_c3b.log 2>&1
rc=$?; tail -1 $OUT/pytest_c3b.log; [ $rc -eq 0 ] || exit $rc
bash tools/c3_ab.sh new prev:AEON_HIP_LIB=aeon_amd/variants/prev.so p17h1:AEON_HIP_REC_PHASES=17,AEON_HIP_REC_HELPERS=1 2>&1 | tee $OUT/c3_ab_jobs.txt
