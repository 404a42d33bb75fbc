mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_jpeg.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/jpeg_tests.log 2>&1
rc=$?; tail -22 gpurun_out/jpeg_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/jpeg_stage.py gpu host > gpurun_out/jpeg_stage.json 2> gpurun_out/jpeg_stage.err || { tail -5 gpurun_out/jpeg_stage.err; exit 1; }
AEON_HIP_JPEG_HUFF_LANES=256 timeout -k 10 200 python tools/jpeg_stage.py gpu >> gpurun_out/jpeg_stage.json 2>> gpurun_out/jpeg_stage.err || { tail -5 gpurun_out/jpeg_stage.err; exit 1; }
cat gpurun_out/jpeg_stage.json
