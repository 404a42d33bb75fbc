#!/bin/bash
# C5 step A/B against variant libraries (tools/build_variants.sh): the C5 parity tests with each
# variant, then tools/c5_run.py three rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  AEON_HIP_LIB="$R/aeon_amd/variants/$v.so" timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_parity.py -k "c5" > gpurun_out/c5ab_$v.log 2>&1 || { tail -20 gpurun_out/c5ab_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/c5ab_$v.log)"
done
for rep in 1 2 3; do
  for v in cur "$@"; do
    lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
    AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/c5_run.py 40 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1
  done
done
