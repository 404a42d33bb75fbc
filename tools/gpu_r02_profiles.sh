#!/bin/bash
# Round-2 profile set: PMC passes (tools/gpu_pmc.sh) for C2, C3 and C5, per-kernel summaries, and
# the C2 traffic file bench.py reads (profiles/traffic_r02.json is copied from the output here).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
for cfg in C2 C3 C5; do
  tools/gpu_pmc.sh $cfg > gpurun_out/pmc_$cfg.txt 2>&1 || { echo "pmc $cfg failed"; cat gpurun_out/pmc_$cfg.txt; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc/$cfg $cfg gpurun_out/traffic_r02.json > gpurun_out/pmc_${cfg}_summary.txt || exit 1
  echo "pmc $cfg ok"
done
