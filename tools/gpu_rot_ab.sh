#!/bin/bash
# rotate_tiles time (rocprof kernel stats) for the current library and each variant given.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp
for v in current "$@"; do
  L=""; [ $v = current ] || L="$R/aeon_amd/variants/$v.so"
  rm -rf gpurun_out/rotab_$v
  AEON_HIP_LIB="$L" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rotab_$v -o run -- python tools/rot_probe.py 20 > gpurun_out/rotab_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/rotab_$v.log; exit 1; }
  echo "$v: $(grep 'rotate' gpurun_out/rotab_$v.log | tail -1) | rotate_tiles avg ns: $(grep rotate_tiles gpurun_out/rotab_$v/run_kernel_stats.csv | cut -d, -f4)"
done
