"""JPEG stage A/B on the GPU box: aeon_hip_decode_jpeg_batch (bench.run_jpeg_stage: 256 records of
aeon's img_2112_70.jpg / flowers.jpg per call) and the JPEG -> C2 decoder (bench.run_e2e_jpeg), with
the GPU entropy decoder (jpeg_huff) and with the host one (AEON_HIP_JPEG_HUFF=host).  One JSON line
per mode.  Usage: python tools/jpeg_stage.py [gpu|host ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

for mode in sys.argv[1:] or ["gpu", "host"]:
    if mode == "host":
        os.environ["AEON_HIP_JPEG_HUFF"] = "host"
    else:
        os.environ.pop("AEON_HIP_JPEG_HUFF", None)
    stage = bench.run_jpeg_stage(A, torch)
    e2e = bench.run_e2e_jpeg(A, C, torch, on_device=True)
    print(json.dumps({"mode": mode, "jpeg_stage": stage, "e2e_device_outputs": e2e}), flush=True)
