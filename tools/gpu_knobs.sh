#!/bin/bash
# kbench (C2 or $CFG) of one library ($LIB, default current) under several knob sets given as arguments.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/knobs.log; : > $out
for knobs in "$@"; do
  echo -n "${LIB:-current} | " >> $out
  AEON_HIP_LIB="${LIB:-}" timeout -k 10 120 python tools/kbench.py ${CFG:-C2} $knobs 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $knobs" >> $out; exit 1; }
done
cat $out
