"""C1 through the product decoder (bench.run_c1_decoder) under alternating AEON_HIP_* settings in one
process (each Decoder creates its own context, which reads the environment): python tools/c1_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

torch.cuda.set_device(0)
for rep in range(2):
    for dyn in ("3", "0"):
        os.environ["AEON_HIP_DYN_TAIL"] = dyn
        r = bench.run_c1_decoder(A, C, torch, 2.0)
        print(f"C1 decoder AEON_HIP_DYN_TAIL={dyn}: {r['value'] / 1e3:.1f} K images/s (windows of {r['decode_size']})", flush=True)
