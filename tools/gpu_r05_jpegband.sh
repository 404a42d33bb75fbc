#!/bin/bash
# Round 5: colour-band height of the JPEG colour pass (AEON_HIP_JPEG_BAND rows per workgroup): JPEG +
# decoder tests, then per band a rocprofv3 kernel-trace of tools/jpeg_stage.py gpu (gpurun_out/r05/jpegband_<b>/).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jpeg.py tests/test_decoder.py > "$O/pytest_jpegband.log" 2>&1
rc=$?; echo "jpeg+decoder tests rc=$rc $(tail -n 1 $O/pytest_jpegband.log)"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for b in 32 16 64 32; do
  rm -rf "$O/jpegband_$b"
  (cd /tmp && AEON_HIP_JPEG_BAND=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/jpegband_$b" -o run --output-format csv -- python3 "$R/tools/jpeg_stage.py" gpu > "$O/jpegband_${b}_prof.log" 2>&1) || exit 1
  f=$(find "$O/jpegband_$b" -name '*kernel_stats.csv' | head -n 1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'jpeg_color' in r['Name'] or 'jpeg_idct' in r['Name']:
        print('band $b', r['Name'][:24], 'calls', r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))"
done
