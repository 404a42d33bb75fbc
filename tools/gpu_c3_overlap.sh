#!/bin/bash
# C3 step time (bench.py --config C3, batch 1024) across the overlap_contrast knobs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/c3_overlap.log
for v in "1 0 0" "2 2 1" "4 2 1" "8 2 1" "4 3 1" "4 2 2" "4 0 0" "8 3 2"; do
  set -- $v
  AEON_HIP_OVERLAP_CHUNKS=$1 AEON_HIP_CAP_PASS1=$2 AEON_HIP_CAP_PASS2=$3 timeout -k 10 120 python bench.py --config C3 --steps 30 --warmup 3 --no-extra --no-cpu-baseline --timing-every 0 2>/dev/null \
    | python -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print('chunks $1 cap1 $2 cap2 $3: %.0f img/s %.1f us/step' % (d['value'], d['ms_per_step']*1e3))" >> gpurun_out/c3_overlap.log || exit 1
done
cat gpurun_out/c3_overlap.log
