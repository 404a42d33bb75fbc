"""Kernel micro-benchmark: per-launch kernel time and HBM rate for C2/C3 under tuning knobs.
Usage: python tools/kbench.py [config] [knob=value ...]  (knobs are AEON_HIP_* env vars)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402


def measure(cfg, batch, steps=20, warmup=3):
    """Per step (one batch): summed kernel time of each kind and its algorithmic-byte rate."""
    torch.cuda.set_device(0)
    _, kt, _, _ = bench.run_device(A, C, torch, cfg, batch, steps, warmup, 0, 1, 400, None, 1,
                                   real=os.environ.get("KBENCH_REAL") == "1")
    res = {}
    for k, (ms, by, n) in kt.items():
        if n:
            res[k] = (ms / n, by / (ms * 1e-3) / 1e9)
    return res


if __name__ == "__main__":
    variants = [dict()]
    cfgs = (("C2", 256), ("C3", 1024))
    argv = sys.argv[1:]
    if argv and argv[0].split(":")[0] in ("C2", "C3"):
        cfgs = ((argv[0], 1024 if argv[0].startswith("C3") else 256),)
        argv = argv[1:]
    if argv == ["default"]:
        variants = [dict()]
    elif argv:
        variants = [dict(kv.split("=", 1) for kv in argv)]
    for cfg, batch in cfgs:
        for v in variants:
            os.environ.update(v)
            r = measure(cfg, batch)
            print(cfg, v, {k: f"{ms*1e3:.1f}us {gbs:.0f}GB/s" for k, (ms, gbs) in r.items()}, flush=True)
