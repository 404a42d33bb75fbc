"""JPEG -> C2 through aeon_decoder alone (bench.run_e2e_jpeg, device outputs), for kernel traces of the
decoder's window pipeline.  Usage: python tools/e2e_jpeg_only.py [windows]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

w = int(sys.argv[1]) if len(sys.argv) > 1 else 30
print("e2e device outputs %.1f K records/s" % (bench.run_e2e_jpeg(A, C, torch, windows=w, on_device=True) / 1e3), flush=True)
