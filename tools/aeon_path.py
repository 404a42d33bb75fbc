"""bench.run_aeon_path alone, with and without the overlap (python tools/aeon_path.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

for cfg in ("C1", "C2"):
    for ov in (True, False, True, False):
        r = bench.run_aeon_path(A, C, torch, cfg, overlap=ov)
        print(json.dumps({"cfg": cfg, "overlap": ov, "value": round(r["value"]), "ms_per_window": round(r["ms_per_window"], 2)}),
              flush=True)
