#!/bin/bash
# PMC A/B of the contrast pass-1 kernel: aeon_amd/variants/old.so against the current library,
# two counter groups each (instruction mix, stalls), summarised per kernel.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
cd /tmp
rm -rf "$R/gpurun_out/pmcab"; mkdir -p "$R/gpurun_out/pmcab"
for lib in old new; do
  L=""; [ $lib = old ] && L="$R/aeon_amd/variants/old.so"
  i=0
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    AEON_HIP_LIB="$L" timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmcab/$lib/p$i" -o run -- python3 "$R/tools/kbench.py" ${CFG:-C3} default > "$R/gpurun_out/pmcab/$lib.p$i.log" 2>&1 || { echo "$lib pass $i failed"; tail -5 "$R/gpurun_out/pmcab/$lib.p$i.log"; exit 1; }
  done
  echo "== $lib"; python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmcab/$lib" | grep -A16 "augment_tiles<1"
done
