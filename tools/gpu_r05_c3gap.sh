#!/bin/bash
# Round 5: C3 launches back to back (untimed) -- kernel trace gaps and the host profile of the call.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python3 -u tools/c3_run.py 30 > "$O/c3_hostprof.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$O/c3_hostprof.txt" | tail -3
(cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$O/c3_trace" -o run -- python3 "$R/tools/c3_run.py" 30 > "$O/c3_trace.log" 2>&1) || exit $?
python3 tools/trace_gaps.py "$O/c3_trace" 30
