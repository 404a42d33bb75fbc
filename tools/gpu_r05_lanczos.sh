#!/bin/bash
# Round 5: LANCZOS4 taps finished on the device (host: anchor, fraction, libm sin/cos only) against
# the previous commit's library (aeon_amd/variants/prev.so: the whole taps on the host): the resize
# GPU tests, then the C2:LANCZOS4 / CUBIC step (tools/interp_steps.py) with each library, twice.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_resize_methods.py tests/test_resize_methods.py > "$O/pytest_lanczos.log" 2>&1
rc=$?; echo "resize tests rc=$rc $(tail -n 1 $O/pytest_lanczos.log)"; [ $rc -eq 0 ] || exit $rc
for lib in new prev new prev; do
  if [ $lib = prev ]; then export AEON_HIP_LIB="$R/aeon_amd/variants/prev.so"; else unset AEON_HIP_LIB; fi
  echo "== $lib"
  timeout -k 10 200 python3 -u tools/interp_steps.py 20 LANCZOS4,CUBIC 2>/dev/null || exit 1
done
