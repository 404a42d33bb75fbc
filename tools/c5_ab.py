"""C5 step and kernel time (bench.run_c5) under the current environment (e.g. AEON_HIP_DIRECT=0/1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    for rep in range(2):
        r = bench.run_c5(A, C, torch, 40, 5, 400)
        print(f"C5 DIRECT={os.environ.get('AEON_HIP_DIRECT', '1')} step {r['ms_per_step'] * 1e3:.1f}us "
              f"kernels {r['kernels_ms_per_step'] * 1e3:.1f}us", flush=True)
