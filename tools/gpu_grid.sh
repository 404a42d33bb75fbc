#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
AEON_HIP_HOST_PROFILE=1 timeout -k 10 120 python tools/kbench.py C2 default 2>&1 | grep -v amdgpu.ids | head -5
