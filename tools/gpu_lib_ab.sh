#!/bin/bash
# Variant libraries (tools/build_variants.sh) A/B: per-launch kernel times (tools/kbench.py CFG) and
# C2 bench lines, twice each.  Usage: CFG=C2 tools/gpu_lib_ab.sh variant...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for v in cur "$@"; do
    lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
    for cfg in ${CFGS:-C2}; do
      echo -n "$v | "; AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/kbench.py $cfg ${KNOBS:-default} 2>&1 | grep -v amdgpu.ids || exit 1
    done
    AEON_HIP_LIB="$lib" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/lab.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/lab.json'))
print('$v bench', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2))"
  done
done
