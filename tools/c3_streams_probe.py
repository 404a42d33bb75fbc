"""C3 across two caller streams (consecutive batches alternate, as aeon's double-buffered output
containers would): with per-CU caps on the two passes' persistent grids (AEON_HIP_CAP_PASS1/2)
batch i's memory-bound pass 2 can share the CUs with batch i+1's VALU-bound pass 1.
Usage: python tools/c3_streams_probe.py  (prints us/step for each setting)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

torch.cuda.set_device(0)
steps = 20
for streams in (1, 2):
    e, _, _, _ = bench.run_device(A, C, torch, "C3", 1024, steps, 3, 0, 1, 400, None, 0, streams)
    print(f"C3 streams={streams} caps=({os.environ.get('AEON_HIP_CAP_PASS1', '-')},"
          f"{os.environ.get('AEON_HIP_CAP_PASS2', '-')}): {e / steps * 1e6:.1f} us/step, "
          f"{1024 * steps / e / 1e6:.2f} M img/s", flush=True)
