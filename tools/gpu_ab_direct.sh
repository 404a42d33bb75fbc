#!/bin/bash
# Kernel times (tools/kbench.py C2) of library variants with the job table in pinned host memory
# (AEON_HIP_DIRECT=1, the default) and uploaded to the device (AEON_HIP_DIRECT=0).
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for rep in 1 2; do
for v in cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="aeon_amd/variants/$v.so"
  for d in 1 0; do echo -n "$v DIRECT=$d "; AEON_HIP_LIB="$lib" AEON_HIP_DIRECT=$d timeout -k 10 120 python tools/kbench.py C2 default 2>&1 | grep -v amdgpu.ids; done
done
done
