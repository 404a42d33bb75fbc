#!/bin/bash
# JPEG stage A/B: GPU tests of the JPEG + decoder paths, then per library variant the stage rate and
# the rocprofv3 kernel stats of jpeg_idct / jpeg_color (tools/jpeg_ab.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg.py tests/test_decoder.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_jpeg.log 2>&1 || { tail -30 gpurun_out/pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/pytest_jpeg.log
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/jpeg_ab.py 2>&1 | grep -v amdgpu.ids || exit 1
  (cd /tmp && AEON_HIP_LIB="$lib" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_jpeg_$v" -o run -- python "$R/tools/jpeg_ab.py" > /dev/null 2>&1) || exit 1
  f=$(find "$R/gpurun_out/prof_jpeg_$v" -name "*kernel_stats.csv" | head -1)
  grep -E "jpeg|Name" "$f" | cut -d, -f1-8
done
