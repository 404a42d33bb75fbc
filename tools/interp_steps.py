"""C2 step time with each interpolation_method (bench.run_device on "C2:<method>", 256 records of
256x256 -> 224x224 fp32, untimed launches): the generic resize pre-pass plus the tile kernel, host
planning included.  Usage: python tools/interp_steps.py [steps] [METHOD,...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for m in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("LINEAR", "CUBIC", "AREA", "LANCZOS4")):
    cfg = "C2" if m == "LINEAR" else "C2:" + m
    e, _, _, _ = bench.run_device(A, C, torch, cfg, 256, steps, 10, 0, 1, 400, None, 0)
    print(f"{m:9s} {e / steps * 1e6:9.1f} us/step  {256 * steps / e:12.0f} img/s", flush=True)
