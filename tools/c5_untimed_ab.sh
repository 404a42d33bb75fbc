#!/bin/bash
# C5 A/B through bench.run_c5 (the bench line's C5 extra: untimed rate), three interleaved rounds per
# case.  A case is name[:VAR=VAL[,VAR=VAL...]].  Usage: tools/c5_untimed_ab.sh base tr48:AEON_HIP_TILE_ROWS=48
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
for round in 1 2 3; do
  for spec in "$@"; do
    name="${spec%%:*}"; envs=""
    [ "$spec" != "$name" ] && envs="${spec#*:}"
    ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 120 python -c "
import torch, bench, aeon_amd as A
from aeon_amd import configs as C
d = bench.run_c5(A, C, torch, 40, 3, 400, kernel_timing=False)
print('$name', round(d['ms_per_step'] * 1e3, 1))" 2>&1 | grep -v amdgpu.ids ) || exit 1
  done
done
