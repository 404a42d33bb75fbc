"""Run bench.py's C5 side workload alone (for rocprofv3 per-kernel stats): python tools/c5_run.py [steps]
(C5_NO_TIMING=1: the untimed run only, for kernel traces of the real schedule)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
print(json.dumps(bench.run_c5(A, C, torch, steps, 10, 400, kernel_timing=os.environ.get("C5_NO_TIMING") != "1")))
