#!/bin/bash
# Round 5: kernel-boundary gaps under rocprofv3 -- C2 contract run (reference) vs C5 pair calls
# (default, fused one-launch form, two separate calls).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
tr() { # name cmd...
  local name=$1; shift
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/gap_$name" -o run -- "$@" > "$O/gap_$name.log" 2>&1) || return $?
  echo "== $name"; python3 tools/trace_gaps.py "$O/gap_$name" 120
}
export C5_NO_TIMING=1; \
  tr c5 python3 "$R/tools/c5_run.py" 50 && \
  AEON_HIP_FUSE_MASKS=1 tr c5fused python3 "$R/tools/c5_run.py" 50 && \
  AEON_BENCH_C5_SEPARATE=1 tr c5sep python3 "$R/tools/c5_run.py" 50
