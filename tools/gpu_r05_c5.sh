#!/bin/bash
# Round 5: where C5's step goes -- kernel trace gaps, host profile of the pair call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python3 -u tools/c5_run.py 50 > "$O/c5_hostprof.txt" 2>&1 || exit $?
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/c5_trace" -o run -- python3 "$R/tools/c5_run.py" 50 > "$O/c5_trace.log" 2>&1) || exit $?
python3 tools/trace_gaps.py "$O/c5_trace" 120 > "$O/c5_gaps.txt"
cat "$O/c5_gaps.txt"; grep -v amdgpu.ids "$O/c5_hostprof.txt" | tail -5
