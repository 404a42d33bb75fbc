#!/bin/bash
# Host-side cost of one bench step on the GPU box: the driver's bench command with the
# per-phase host profile (AEON_HIP_HOST_PROFILE=1), at the driver's step count and at 200.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt; grep -m1 "model name" /proc/cpuinfo >> gpurun_out/nproc.txt
python -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >> gpurun_out/nproc.txt
for steps in 20 200; do
  AEON_HIP_HOST_PROFILE=1 timeout -k 10 180 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --no-extra \
    > gpurun_out/hostprof_$steps.log 2> gpurun_out/hostprof_$steps.err || { echo "bench $steps failed"; tail -5 gpurun_out/hostprof_$steps.err; exit 1; }
done
cat gpurun_out/nproc.txt
for steps in 20 200; do tail -1 gpurun_out/hostprof_$steps.log; grep "host profile" gpurun_out/hostprof_$steps.err; done
