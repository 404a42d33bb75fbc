#!/bin/bash
# C2 contract-line repeatability: direct calls vs the device-job-table path, and the host phases.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/direct_check.log; : > $out
summ() { python -c "
import json,sys; d=json.load(open('$1'))
print('$2', round(d['value']), 'img/s', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_launch_ms']*1e3,2), 'submit', round(d['host_submit_ms_per_step']*1e3,2), 'us')" >> $out; }
for rep in 1 2; do
  for dm in 1 0; do
    AEON_HIP_DIRECT=$dm timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/dc_$dm.json 2>gpurun_out/dc_$dm.err || { tail -5 gpurun_out/dc_$dm.err; exit 1; }
    summ gpurun_out/dc_$dm.json "direct=$dm 20 steps"
  done
done
for dm in 1 0; do
  AEON_HIP_DIRECT=$dm timeout -k 10 120 python bench.py --steps 200 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/dc_$dm.json 2>gpurun_out/dc_$dm.err || exit 1
  summ gpurun_out/dc_$dm.json "direct=$dm 200 steps"
  AEON_HIP_HOST_PROFILE=1 AEON_HIP_DIRECT=$dm timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > /dev/null 2>gpurun_out/dc_prof_$dm.err || exit 1
  grep -v amdgpu.ids gpurun_out/dc_prof_$dm.err | tail -12 >> $out
done
cat $out
