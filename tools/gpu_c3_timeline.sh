#!/bin/bash
# Where a C3 step's time goes: host planning profile (AEON_HIP_HOST_PROFILE=1) and a rocprofv3
# kernel trace of the same bench run, reduced to per-kernel durations and the gaps between them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AEON_HIP_HOST_PROFILE=1 timeout -k 10 180 python bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-extra \
  > gpurun_out/c3tl_bench.log 2> gpurun_out/c3tl_bench.err || { echo "bench failed"; tail -5 gpurun_out/c3tl_bench.err; exit 1; }
tail -1 gpurun_out/c3tl_bench.log | cut -c1-400
grep "host profile" -A8 gpurun_out/c3tl_bench.err
rm -rf gpurun_out/c3tl
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3tl -- python bench.py --config C3 --steps 50 --warmup 5 --no-cpu-baseline --no-extra \
  > gpurun_out/c3tl_prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/c3tl_prof.log; exit 1; }
python tools/trace_gaps.py gpurun_out/c3tl 300
