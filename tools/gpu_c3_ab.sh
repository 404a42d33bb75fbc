#!/bin/bash
# C3 step A/B: bench.py --config C3 against variant libraries (tools/build_variants.sh), three rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in cur "$@"; do
    lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
    AEON_HIP_LIB="$lib" timeout -k 10 180 python bench.py --config C3 --steps 30 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/c3ab.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/c3ab.json'))
print('$v C3', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,1), 'us/step', d['config'].get('global_batch'), {k: round(v*1e3,1) if isinstance(v,float) else v for k,v in d['roofline'].items() if 'ms' in k})"
  done
done
