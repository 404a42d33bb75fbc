#!/bin/bash
# Round 6: augment_split (staging helper waves) -- GPU tests, then the C2 A/B against augment_tiles.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
OUT=gpurun_out/r06; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/c2_ab.sh split:AEON_HIP_SPLIT=1 tiles:AEON_HIP_SPLIT=0 split3:AEON_HIP_SPLIT=1,AEON_HIP_SPLIT_RPL=3 2>&1 | tee $OUT/c2_split_ab.txt
for cfg in C2 C1; do for b in pinned pageable; do for m in overlap flush; do
  timeout -k 10 120 ./aeon_amd/aeon_path_cpp $cfg $b $m 16 3 | tee -a $OUT/aeon_path_cpp.txt || exit 1
done; done; done
