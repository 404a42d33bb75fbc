#!/bin/bash
# Round 5: where the C2:LANCZOS4 step goes -- host phases (AEON_HIP_HOST_PROFILE=1) per library and a
# rocprofv3 kernel trace of the new one (gpurun_out/r05/lanczos_prof/).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_resize_methods.py tests/test_resize_methods.py > "$O/pytest_lanczos.log" 2>&1
rc=$?; echo "resize tests rc=$rc $(tail -n 1 $O/pytest_lanczos.log)"; [ $rc -eq 0 ] || exit $rc
for lib in new prev; do
  if [ $lib = prev ]; then export AEON_HIP_LIB="$R/aeon_amd/variants/prev.so"; else unset AEON_HIP_LIB; fi
  echo "== $lib"
  AEON_HIP_HOST_PROFILE=1 timeout -k 10 200 python3 -u tools/interp_steps.py 20 LANCZOS4 2>&1 | grep -v amdgpu.ids || exit 1
done
unset AEON_HIP_LIB
rm -rf "$O/lanczos_prof"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/lanczos_prof" -o run --output-format csv -- python3 "$R/tools/interp_steps.py" 20 LANCZOS4 > "$O/lanczos_prof.log" 2>&1) || exit 1
python3 -c "
import csv
rows=sorted(csv.DictReader(open('$O/lanczos_prof/run_kernel_stats.csv')), key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:6]: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
