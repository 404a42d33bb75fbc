#!/bin/bash
# augment_rows ablations (tools/build_variants.sh builds): kernel time of each variant library.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="aeon_amd/variants/$v.so"
  echo -n "$v | "; AEON_HIP_LIB="$lib" timeout -k 10 120 python tools/kbench.py C2 ${KNOBS:-default} 2>&1 | grep -v amdgpu.ids || exit 1
done
