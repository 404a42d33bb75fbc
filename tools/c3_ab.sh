#!/bin/bash
# C3 A/B: tools/c3_run.py (40 untimed steps) per case, three rounds interleaved.  A case is
# name[:VAR=VAL[,VAR=VAL...]] (AEON_HIP_LIB=aeon_amd/variants/<v>.so picks a tools/build_variants.sh build).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
for round in 1 2 3; do
  for spec in "$@"; do
    name="${spec%%:*}"; envs=""
    [ "$spec" != "$name" ] && envs="${spec#*:}"
    r=$( ( IFS=','; for kv in $envs; do export "$kv"; done
      timeout -k 10 120 python tools/c3_run.py 40 2>/dev/null | tail -1 ) ) || exit 1
    echo "$name $r"
  done
done
