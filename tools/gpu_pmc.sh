#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains besides kernel-trace).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/pmc"
export TMPDIR=/tmp
cd /tmp
CFG=${1:-C2}
if [ "$CFG" = C5 ]; then PROG=("$R/tools/c5_run.py" 20); else PROG=("$R/tools/kbench.py" $CFG ${KNOBS:-default}); fi
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmc/$CFG/p$i" -o run -- python3 "${PROG[@]}" > "$R/gpurun_out/pmc/$CFG.p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc/$CFG.p$i.log"; exit 1; }
  echo "pass $i ok"
done
