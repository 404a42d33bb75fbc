#!/bin/bash
# Column-strided lanes A/B: GPU tests, C2 kernel / bench lines (in-tree vs the AEON_HIP_STRIDED=0
# variant), C5 rate, and the LDS counters of the C2 kernel for both.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_lib_ab.sh contig || exit 1
for v in cur contig; do
  lib=""; [ "$v" != cur ] && lib="$R/aeon_amd/variants/$v.so"
  for i in 1 2; do AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/c5_run.py 50 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v C5', round(d['value']), 'pairs/s', round(d['ms_per_step']*1e3,1), 'us/step kernels', round(d['kernels_ms_per_step']*1e3,1))" || exit 1; done
  (cd /tmp && AEON_HIP_LIB="$lib" timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_lds_$v" -o run -- python3 "$R/tools/kbench.py" C2 default > "$R/gpurun_out/pmc_lds_$v.log" 2>&1) || exit 1
  python tools/pmc_summary.py gpurun_out/pmc_lds_$v C2 | grep -A5 "augment_tiles"
done
