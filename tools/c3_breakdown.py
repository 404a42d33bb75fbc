"""C3 cost breakdown: contrast pass 1 (STATS) and pass 2 kernel times with photometric stages
switched off one at a time (development tool; the stages' order and arithmetic are unchanged)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

VARIANTS = {
    "full C3": {},
    "no hue": {"hue": [0, 0]},
    "no saturation (diag transform)": {"saturation": [1.0, 1.0]},
    "no hue, no saturation": {"hue": [0, 0], "saturation": [1.0, 1.0]},
    "contrast only": {"hue": [0, 0], "saturation": [1.0, 1.0], "brightness": [1.0, 1.0], "lighting": [0.0, 0.0]},
}

if __name__ == "__main__":
    # optional knob sets: python tools/c3_breakdown.py "AEON_HIP_WG_PER_CU=2" "AEON_HIP_THREADS=256" ...
    knobs = [dict()] + [dict(kv.split("=", 1) for kv in arg.split(",")) for arg in sys.argv[1:]]
    torch.cuda.set_device(0)
    base = dict(C.C3_AUG)
    for kn in knobs:
        for k in ("AEON_HIP_WG_PER_CU", "AEON_HIP_THREADS", "AEON_HIP_TR", "AEON_HIP_STAGE_KB"):
            os.environ.pop(k, None)
        os.environ.update(kn)
        for name, over in VARIANTS.items():
            if kn and name not in ("full C3", "contrast only"):
                continue
            C.C3_AUG = dict(base, **over)
            _, kt, _, _ = bench.run_device(A, C, torch, "C3", 1024, 20, 3, 0, 1, 400, None, 1)
            res = {k: f"{ms / n * 1e3:.1f}us" for k, (ms, by, n) in kt.items() if n}
            print(f"{str(kn):40s} {name:34s} {res}", flush=True)
