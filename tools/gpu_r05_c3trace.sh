#!/bin/bash
# Round 5: the C3 record kernel's per-phase trace (noise and real sources), its kernel time on both
# sources, and the LDS bank-conflict counters on both.  Outputs under gpurun_out/r05/.
set -eo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r05"
mkdir -p "$O"
cd "$R"
AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 180 python3 -u tools/trace_records.py > "$O/trace_c3_noise.txt" 2>&1
AEON_HIP_LIB=aeon_amd/variants/trace.so timeout -k 10 180 python3 -u tools/trace_records.py real > "$O/trace_c3_real.txt" 2>&1
timeout -k 10 180 python3 -u tools/kbench.py C3 > "$O/kbench_c3_noise.txt" 2>&1
KBENCH_REAL=1 timeout -k 10 180 python3 -u tools/kbench.py C3 > "$O/kbench_c3_real.txt" 2>&1
export TMPDIR=/tmp
for src in noise real; do
  if [ $src = real ]; then export KBENCH_REAL=1; else unset KBENCH_REAL; fi
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --kernel-trace --output-format csv -d "$O/pmc_c3_$src" -o run -- python3 "$R/tools/kbench.py" C3 > "$O/pmc_c3_$src.log" 2>&1)
done
echo done
