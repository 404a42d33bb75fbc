#!/bin/bash
# A/B: current library vs aeon_amd/variants/*.so, C2 per-step kernel time under staging knobs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
out=gpurun_out/ab.log; : > $out
run() { echo -n "$1 | " >> $out; AEON_HIP_LIB="$2" timeout -k 10 120 python tools/kbench.py ${CFG:-C2} $3 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $1 $3" >> $out; return 1; }; }
run old aeon_amd/variants/old.so default && run old aeon_amd/variants/old.so "AEON_HIP_TR=16 AEON_HIP_BANDS=1" || exit 1
for knobs in default "AEON_HIP_THREADS=256" "AEON_HIP_THREADS=384" "AEON_HIP_THREADS=512" "AEON_HIP_TR=8" "AEON_HIP_THREADS=256 AEON_HIP_TR=8" "AEON_HIP_THREADS=512 AEON_HIP_TR=18" "AEON_HIP_BANDS=2"; do
  run new "" "$knobs" || exit 1
done
cat $out
