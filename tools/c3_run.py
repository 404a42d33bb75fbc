"""bench.py's C3 side workload alone, untimed launches (for kernel traces of the real schedule):
python tools/c3_run.py [steps]."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
torch.cuda.set_device(0)
e, _, _, _ = bench.run_device(A, C, torch, "C3", 1024, steps, 5, 0, 1, 400, None, 0)
print(f"C3 {e / steps * 1e6:.1f} us/step")
