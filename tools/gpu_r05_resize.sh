#!/bin/bash
# Round 5: the LDS-staged resize_generic -- its parity tests, step times per interpolation method,
# rocprof kernel stats of the CUBIC workload.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_resize_methods.py > "$O/pytest_resize.log" 2>&1
rc=$?; echo "resize tests rc=$rc $(tail -n 1 $O/pytest_resize.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/interp_steps.py 20 2>&1 | grep -v amdgpu.ids | tee "$O/interp_steps.txt"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_cubic" -o run --output-format csv -- python3 "$R/tools/kbench.py" C2:CUBIC default > "$O/prof_cubic.log" 2>&1) || exit 1
python3 - "$O/prof_cubic/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "aeon" in r["Name"]:
        print("%-60s n=%5s avg=%8.2f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
