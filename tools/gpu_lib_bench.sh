#!/bin/bash
# bench.py step rate (C2, one stream, no timing events) for the current library and each
# aeon_amd/variants/<name>.so given as arguments (development A/B of whole steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
out=gpurun_out/lib_bench.log; : > $out
for v in current "$@"; do
  lib=""; [ "$v" != current ] && lib=aeon_amd/variants/$v.so
  echo -n "$v | " >> $out
  AEON_HIP_LIB="$lib" timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-extra \
    --timing-every ${EVERY:-0} --streams ${STREAMS:-1} 2>/dev/null \
    | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); r=d['roofline']; print('value %.0f ms/step %.4f kernel_ms %.4f' % (d['value'], d['ms_per_step'], r['kernel_avg_launch_ms']))" >> $out \
    || { echo FAILED >> $out; exit 1; }
done
cat $out
