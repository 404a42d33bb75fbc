#!/bin/bash
# Host-side cost of one augment_batch call (per-phase, AEON_HIP_HOST_PROFILE) next to the bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AEON_HIP_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-extra \
  > gpurun_out/hostprof.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/hostprof.log
exit $rc
