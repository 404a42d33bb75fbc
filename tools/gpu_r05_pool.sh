#!/bin/bash
# Round 5: LANCZOS4 taps finished on the device + thread_pool runs that wait for their tasks rather than
# for every worker, against the previous commit's library (aeon_amd/variants/prev.so): GPU tests of the
# pool's users, then per library (twice, alternating) the C2:LANCZOS4 step with host phases
# (AEON_HIP_HOST_PROFILE=1), the JPEG stage and the C1 decoder.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_resize_methods.py tests/test_resize_methods.py tests/test_decoder.py tests/test_jpeg.py tests/test_integration.py > "$O/pytest_pool.log" 2>&1
rc=$?; echo "tests rc=$rc $(tail -n 1 $O/pytest_pool.log)"; [ $rc -eq 0 ] || exit $rc
for lib in new prev new prev; do
  if [ $lib = prev ]; then export AEON_HIP_LIB="$R/aeon_amd/variants/prev.so"; else unset AEON_HIP_LIB; fi
  echo "== $lib"
  AEON_HIP_HOST_PROFILE=1 timeout -k 10 200 python3 -u tools/interp_steps.py 20 LANCZOS4 2>&1 | grep -E "host profile|us/step" | sed -e 's/.*host profile\]/  host/' || exit 1
  timeout -k 10 200 python3 -u tools/jpeg_stage.py gpu 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['jpeg_stage']; e=d['e2e_device_outputs']
print('  jpeg stage %.1f K  e2e %.1f K' % (s['value']/1e3, (e['value'] if isinstance(e,dict) else e)/1e3))" || exit 1
done
