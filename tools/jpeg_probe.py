"""JPEG stage kernel time per window shape (development probe for jpeg_huff / jpeg_bands): the
kernels' HIP-event time (ctx.kernel_times()["jpeg"]: jpeg_huff + the pixel kernels) for windows of
one file repeated, with the GPU entropy decoder and with the host one (AEON_HIP_JPEG_HUFF=host: the
pixel kernels alone).  One line per (mode, window).  Usage: python tools/jpeg_probe.py [n ...]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import aeon_amd as A  # noqa: E402

FX = np.load(os.path.join(ROOT, "tests", "golden", "jpeg_fixtures.npz"))


def kernel_us(ctx, files, reps=8):
    infos = [A.jpeg_info(f) for f in files]
    descs, off = [], 0
    for (w, h, _) in infos:
        descs.append(A.ImgDesc(offset=off, width=w, height=h, stride=w * 3, channels=3))
        off += (w * h * 3 + 15) // 16 * 16
    descs = (A.ImgDesc * len(files))(*descs)
    dst = torch.empty(off, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        ctx.decode_jpeg_batch(files, descs, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    ctx.kernel_times()
    ctx.set_timing(1)
    for _ in range(reps):
        ctx.decode_jpeg_batch(files, descs, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    ms, _, n = ctx.kernel_times()["jpeg"]
    ctx.set_timing(False)
    return ms * 1e3 / max(n, 1)


counts = [int(a) for a in sys.argv[1:]] or [1, 256]
for mode in (("gpu",) if os.environ.get("JPEG_PROBE_GPU_ONLY") else ("gpu", "host")):
    if mode == "host":
        os.environ["AEON_HIP_JPEG_HUFF"] = "host"
    ctx = A.Context(0)
    for name in ("img_2112_70", "flowers", "s420_q50", "q100"):
        f = FX[name + ".jpg"].tobytes()
        for n in counts:
            print(f"{mode:4s} {name:12s} x{n:<4d} {kernel_us(ctx, [f] * n):9.1f} us per call", flush=True)
    ctx.close()
