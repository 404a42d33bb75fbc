#!/bin/bash
# Round 5: the JPEG pixel kernels (jpeg_idct range limit, jpeg_color 4:2:0 path) against the previous
# commit's library (aeon_amd/variants/prev.so, built from `git archive HEAD` by hand): JPEG + decoder
# tests, then per library the stage numbers (tools/jpeg_stage.py gpu) and a rocprofv3 kernel-trace
# of the same command (per-kernel stats into gpurun_out/r05/jpegpix_<lib>/).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jpeg.py tests/test_decoder.py > "$O/pytest_jpegpix.log" 2>&1
rc=$?; echo "jpeg+decoder tests rc=$rc $(tail -n 1 $O/pytest_jpegpix.log)"; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for lib in new prev new2 prev2; do
  if [ ${lib%2} = prev ]; then export AEON_HIP_LIB="$R/aeon_amd/variants/prev.so"; else unset AEON_HIP_LIB; fi
  timeout -k 10 200 python3 -u tools/jpeg_stage.py gpu 2>/dev/null > "$O/jpegpix_$lib.json" || exit 1
  python3 -c "
import json; d = json.loads(open('$O/jpegpix_$lib.json').read().strip().splitlines()[-1])
s = d['jpeg_stage']; e = d['e2e_device_outputs']
ev = e['value'] if isinstance(e, dict) else e
print('$lib stage %.1f K img/s gpu %.2f us/rec  e2e %.1f K' % (s['value'] / 1e3, s['gpu_us_per_record'], ev / 1e3))"
  rm -rf "$O/jpegpix_$lib"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/jpegpix_$lib" -o run --output-format csv -- python3 "$R/tools/jpeg_stage.py" gpu > "$O/jpegpix_${lib}_prof.log" 2>&1) || exit 1
  f=$(find "$O/jpegpix_$lib" -name '*kernel_stats.csv' | head -n 1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'jpeg' in r['Name']:
        print('$lib', r['Name'][:40], 'calls', r['Calls'], 'avg %.1f us' % (float(r['AverageNs']) / 1e3))"
done
