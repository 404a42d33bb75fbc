#!/bin/bash
# Round 5: resize_sep (register-window separable resize) -- parity tests, step times, rocprof stats
# at band heights 32 / 16.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_resize_methods.py > "$O/pytest_resize.log" 2>&1
rc=$?; echo "resize tests rc=$rc $(tail -n 1 $O/pytest_resize.log)"; [ $rc -eq 0 ] || exit $rc
for tr in 16; do unset AEON_HIP_SEP_TR;
  echo "== band rows $tr"
  AEON_HIP_SEP_TR=$tr timeout -k 10 300 python3 -u tools/interp_steps.py 20 2>&1 | grep -v amdgpu.ids
  (cd /tmp && AEON_HIP_SEP_TR=$tr timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_cubic_$tr" -o run --output-format csv -- python3 "$R/tools/kbench.py" C2:CUBIC default > "$O/prof_cubic_$tr.log" 2>&1) || exit 1
  python3 - "$O/prof_cubic_$tr/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "aeon" in r["Name"]:
        print("%-60s n=%5s avg=%8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
