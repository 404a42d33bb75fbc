#!/bin/bash
# C5 step A/B: tools/c5_run.py (50 steps) per case, each twice, interleaved.  A case is
# name[:VAR=VAL[,VAR=VAL...]] -- environment for that run (AEON_HIP_LIB=aeon_amd/variants/<v>.so picks a
# tools/build_variants.sh build; AEON_BENCH_C5_SEPARATE=1 = the image and mask calls of round 4;
# AEON_HIP_FUSE_MASKS=1 = the one-launch form).
# Usage: tools/c5_ab.sh pair calls:AEON_BENCH_C5_SEPARATE=1 fused:AEON_HIP_FUSE_MASKS=1
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
for round in 1 2; do
  for spec in "$@"; do
    name="${spec%%:*}"; envs=""
    [ "$spec" != "$name" ] && envs="${spec#*:}"
    ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 120 python tools/c5_run.py 50 > "gpurun_out/c5_$name.json" ) || exit 1
    python -c "import json;d=json.load(open('gpurun_out/c5_$name.json'));print('$name', round(d['ms_per_step']*1e3,1), round(d.get('kernels_ms_per_step',0)*1e3,1))"
  done
done
