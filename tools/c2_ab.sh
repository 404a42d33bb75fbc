#!/bin/bash
# C2 A/B: bench.py's contract run (200 steps, no extras) per case, each three times, interleaved.  A case
# is name[:VAR=VAL[,VAR=VAL...]] (AEON_HIP_LIB=aeon_amd/variants/<v>.so picks a tools/build_variants.sh
# build).  Prints ms_per_step and the dominant kernel's event-timed duration.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
for round in 1 2 3; do
  for spec in "$@"; do
    name="${spec%%:*}"; envs=""
    [ "$spec" != "$name" ] && envs="${spec#*:}"
    ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-extra > "gpurun_out/c2_$name.json" ) || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/c2_$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', 'step_us', round(d['ms_per_step']*1e3,2), 'kernel_us', round(r['kernel_avg_launch_ms']*1e3,2), 'frac', round(r['frac'],4))"
  done
done
