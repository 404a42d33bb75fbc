#!/bin/bash
# C3 with both contrast passes in one launch (augment_contrast_fused) against the three-launch
# schedule: parity first, then bench.py --config C3 per setting (ms/step, kernel time).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_parity.py tests/test_decoder.py \
  -m gpu -k "${TESTS:-c3 or C3 or contrast or full_batch or edge or decoder or device_planner or overlap}" > gpurun_out/t_fused.log 2>&1 \
  || { tail -30 gpurun_out/t_fused.log; exit 1; }
tail -1 gpurun_out/t_fused.log
for v in ${VARIANTS:-"AEON_HIP_FUSED=0" "AEON_HIP_FUSED=1" "AEON_HIP_FUSED_LAG=64" "AEON_HIP_FUSED_LAG=192"}; do
  env $v timeout -k 10 120 python bench.py --config C3 --steps 50 --warmup 5 --no-extra --no-cpu-baseline 2>/dev/null \
    | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); r=d['roofline']; print('$v value %.0f ms/step %.4f kernel_ms %.4f' % (d['value'], d['ms_per_step'], r['kernel_avg_launch_ms']))" || exit 1
done
