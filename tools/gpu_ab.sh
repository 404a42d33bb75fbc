#!/bin/bash
# Parity tests, then A/B: current library vs aeon_amd/variants/old.so (C2/C3 per-step kernel time),
# plus knob variants of the current library given as arguments ("AEON_HIP_TR=8 AEON_HIP_WG_PER_CU=2" ...).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/ab.log; : > $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
run() { echo -n "$1 | " >> $out; AEON_HIP_LIB="$2" timeout -k 10 120 python tools/kbench.py ${CFG:-C2} $3 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $1 $3" >> $out; return 1; }; }
[ -f aeon_amd/variants/old.so ] && { run old aeon_amd/variants/old.so default || exit 1; }
run new "" default || exit 1
for knobs in "$@"; do run new "" "$knobs" || exit 1; done
cat $out
