#!/bin/bash
# Round 5: JPEG stage with the staging H2D on a copy stream (default) vs on the call's stream
# (AEON_HIP_JPEG_COPY_STREAM=0): JPEG + decoder tests, then tools/jpeg_stage.py gpu twice each.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jpeg.py tests/test_decoder.py > "$O/pytest_jpegcopy.log" 2>&1
rc=$?; echo "jpeg+decoder tests rc=$rc $(tail -n 1 $O/pytest_jpegcopy.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in 1 0; do
    AEON_HIP_JPEG_COPY_STREAM=$m timeout -k 10 200 python3 -u tools/jpeg_stage.py gpu 2>/dev/null > "$O/jpegcopy_$m.json" || exit 1
    python3 -c "
import json; d = json.loads(open('$O/jpegcopy_$m.json').read().strip().splitlines()[-1])
s = d['jpeg_stage']; e = d['e2e_device_outputs']
ev = e['value'] if isinstance(e, dict) else e
print('copy_stream=$m stage %.1f K img/s gpu %.2f us/rec  e2e %.1f K' % (s['value'] / 1e3, s['gpu_us_per_record'], ev / 1e3))"
  done
done
