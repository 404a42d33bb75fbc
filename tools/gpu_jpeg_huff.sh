#!/bin/bash
# JPEG stage on the GPU box: the JPEG tests (GPU entropy decoder vs host, goldens, oracle), then tools/jpeg_stage.py A/B runs -> gpurun_out/jpeg_stage.json, and a
# rocprofv3 kernel summary of the default stage -> gpurun_out/jpeg_prof.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_jpeg.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/jpeg_tests.log 2>&1
rc=$?; tail -24 gpurun_out/jpeg_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/jpeg_stage.py gpu host > gpurun_out/jpeg_stage.json 2> gpurun_out/jpeg_stage.err || { tail -5 gpurun_out/jpeg_stage.err; exit 1; }
AEON_HIP_JPEG_HUFF_LANES=256 timeout -k 10 200 python tools/jpeg_stage.py gpu >> gpurun_out/jpeg_stage.json 2>> gpurun_out/jpeg_stage.err || { tail -5 gpurun_out/jpeg_stage.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/jpeg_stage.json"):
    d = json.loads(l); s = d["jpeg_stage"]
    print(d["mode"], "stage", round(s["value"]), "img/s  gpu us/rec", round(s["gpu_us_per_record"] or 0, 2),
          "host us/file", {k: round(v, 1) for k, v in s["host_stage_us_per_file"].items()}, "e2e", round(d["e2e_device_outputs"]))
PY
rm -rf gpurun_out/jpeg_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jpeg_prof -o run -- python tools/jpeg_stage.py gpu > gpurun_out/jpeg_prof.log 2>&1 || { tail -5 gpurun_out/jpeg_prof.log; exit 1; }
f=$(find gpurun_out/jpeg_prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
