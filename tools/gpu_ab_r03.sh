#!/bin/bash
# Round-3 kernel A/B: parity of each variant library (C2/C5 full batches + the edge cases), then
# per-launch kernel times (tools/kbench.py) of the in-tree library and each variant, twice, and a
# phase trace of the in-tree C2 kernel.  Usage: tools/gpu_ab_r03.sh variant...
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
out=gpurun_out/ab_r03.log; : > $out
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="aeon_amd/variants/$v.so"
  AEON_HIP_LIB="$lib" timeout -k 10 300 python -u -m pytest tests/test_hip_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "full_batch_c2 or full_batch_c5 or edge_cases or golden or configs_fixed or grayscale or padding or zero_copy or rotation_configs or output_types" > gpurun_out/ab_pytest_$v.log 2>&1 \
    || { echo "PARITY FAILED $v: $(tail -1 gpurun_out/ab_pytest_$v.log)" >> $out; }
  echo "parity ok $v: $(tail -1 gpurun_out/ab_pytest_$v.log)" >> $out
done
for rep in 1 2; do
  for v in cur "$@"; do
    lib=""; [ "$v" != cur ] && lib="aeon_amd/variants/$v.so"
    for cfg in ${CFGS:-C2 C3}; do
      echo -n "$v $cfg | " >> $out
      AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/kbench.py $cfg default 2>&1 | grep -v amdgpu.ids >> $out || { echo "FAILED $v" >> $out; exit 1; }
    done
  done
done
timeout -k 10 120 python tools/trace_kernel.py C2 > gpurun_out/trace_c2.log 2>&1 || echo "trace failed" >> $out
cat $out
