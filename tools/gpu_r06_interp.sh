#!/bin/bash
# Round 6: resize_sep (CUBIC / LANCZOS4 / INTER_AREA's bilinear emulation) A/B against aeon_amd/variants/prev.so:
# the resize-method parity tests, then interpolation steps for both libraries, twice, and a kernel-stats pass.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT; T=${1:-x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_resize_methods.py > $OUT/pytest_interp_$T.log 2>&1
rc=$?; tail -1 $OUT/pytest_interp_$T.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in ${VARIANTS:-new noarea prev}; do
    unset AEON_HIP_LIB AEON_HIP_AREA_SEP AEON_HIP_IDENTITY_SEP
    [ $v != new ] && [ -f aeon_amd/variants/$v.so ] && export AEON_HIP_LIB=aeon_amd/variants/$v.so
    [ $v = noarea ] && export AEON_HIP_AREA_SEP=0
    [ $v = noident ] && export AEON_HIP_IDENTITY_SEP=0
    echo "== $v" | tee -a $OUT/interp_$T.txt
    timeout -k 10 200 python tools/interp_steps.py 20 ${METHODS:-CUBIC,AREA,LANCZOS4} 2>&1 | grep -v amdgpu.ids | tee -a $OUT/interp_$T.txt || exit 1
  done
done
unset AEON_HIP_LIB AEON_HIP_AREA_SEP AEON_HIP_IDENTITY_SEP
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_interp_$T -o run --output-format csv -- python tools/interp_steps.py 20 CUBIC,AREA,LANCZOS4 > /dev/null 2>&1 || exit 1
find $OUT/prof_interp_$T -name "*kernel_stats.csv" -exec cp {} $OUT/interp_${T}_kernel_stats.csv \;
python - <<PY
import csv
for r in csv.DictReader(open("$OUT/interp_${T}_kernel_stats.csv")):
    if "aeon" in r["Name"]: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3, 1))
PY
