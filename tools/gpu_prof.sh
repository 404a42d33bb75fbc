#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (args: output name, then bench.py args).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=$1; shift
mkdir -p "$R/gpurun_out/$name"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/$name" -o run --output-format csv -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/$name/bench.log" 2>&1 || { tail -5 "$R/gpurun_out/$name/bench.log"; exit 1; }
f=$(find "$R/gpurun_out/$name" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12
