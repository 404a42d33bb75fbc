#!/bin/bash
# C5 mask gather A/B: rocprofv3 kernel stats of the C5 workload with the staged gather (rows per
# workgroup swept) and the direct gather.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c5_$name -o c5 --output-format csv -- \
    python tools/c5_run.py 100 > gpurun_out/c5_$name.log 2>&1 || exit 1
  echo "== $name: $(grep '^{' gpurun_out/c5_$name.log | cut -c1-120)"
  find gpurun_out/c5_$name -name '*kernel_stats.csv' -exec cat {} \; | cut -d, -f1-8 | grep -i "nearest\|Name"
}
run staged AEON_HIP_MASK_GATHER=staged
run direct AEON_HIP_MASK_GATHER=direct
run noperm AEON_HIP_MASK_PERM=0
for r in 32; do run staged_r$r AEON_HIP_NEAREST_ROWS=$r; done
