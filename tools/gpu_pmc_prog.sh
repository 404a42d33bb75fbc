#!/bin/bash
# Two PMC passes (instruction mix / stalls) over any python program, summarised for kernels whose
# name matches $KERNEL: tools/gpu_pmc_prog.sh <kernel-substring> <script.py> [args]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
K="$1"; shift
rm -rf "$R/gpurun_out/pmcprog"; mkdir -p "$R/gpurun_out/pmcprog"
cd /tmp
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmcprog/p$i" -o run -- python3 "$R/$@" > "$R/gpurun_out/pmcprog/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmcprog/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmcprog" | grep -A18 "$K"
