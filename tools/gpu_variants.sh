#!/bin/bash
# kbench (C2) for the current library and each aeon_amd/variants/<name>.so given as arguments.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/variants.log; : > $out
run() { echo -n "$1 | " >> $out; AEON_HIP_LIB="$2" timeout -k 10 120 python tools/kbench.py ${CFG:-C2} ${KNOBS:-default} 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $1" >> $out; return 1; }; }
run current "" || exit 1
for v in "$@"; do run $v aeon_amd/variants/$v.so || exit 1; done
cat $out
