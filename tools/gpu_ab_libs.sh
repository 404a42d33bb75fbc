#!/bin/bash
# Kernel micro-benchmark (tools/kbench.py) of several library builds on one box: the in-tree library
# ("cur") and each aeon_amd/variants/<name>.so given as an argument.  CFG=C2|C3.  No parity tests.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/ab_libs.log; : > $out
run() { echo -n "$1 | " >> $out; AEON_HIP_LIB="$2" timeout -k 10 120 python tools/kbench.py ${CFG:-C3} default 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $1" >> $out; return 1; }; }
for rep in 1 2; do
  run cur "" || exit 1
  for v in "$@"; do run "$v" "aeon_amd/variants/$v.so" || exit 1; done
done
cat $out
