#!/bin/bash
# C3 over two caller streams with and without per-CU caps on the two passes (tools/c3_streams_probe.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; out=gpurun_out/c3_streams.log; : > $out
p() { env "$@" timeout -k 10 120 python tools/c3_streams_probe.py 2>&1 | grep "C3 streams" >> $out; }
p AEON_HIP_CAPS=0 && p AEON_HIP_CAPS=1 AEON_HIP_CAP_PASS1=2 AEON_HIP_CAP_PASS2=1 \
  && p AEON_HIP_CAPS=1 AEON_HIP_CAP_PASS1=2 AEON_HIP_CAP_PASS2=2 && p AEON_HIP_CAPS=1 AEON_HIP_CAP_PASS1=1 AEON_HIP_CAP_PASS2=1
cat $out
