"""Per-step time of C2 with and without image::rotate (angle drawn from [-15, 15]) on 256 records of
256x256 -> 224x224 fp32 CHW, device-resident: what the rotation pre-pass costs.
Development probe: python tools/rot_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
from aeon_amd import configs as C  # noqa: E402


def run(aug, steps, n=256):
    ctx = A.Context(0)
    w = h = 256
    imgs = [A.synthetic_image(i, w, h, 3) for i in range(n)]
    arena, descs = A.pack_images(imgs)
    src = torch.from_numpy(arena).to("cuda")
    out = C.out_desc_for(C.IMAGE_224, aug)
    dst = torch.empty(n * out.item_stride, dtype=torch.uint8, device="cuda")
    f = A.ParamFactory(aug)
    states = A.seed_slots(1, n)
    params = (A.AugParams * n)(*[f.make_params(states[i:i + 1], w, h, 224, 224) for i in range(n)])
    stream = torch.cuda.current_stream().cuda_stream
    for _ in range(3):
        ctx.augment_batch(descs, src.data_ptr(), params, out, dst.data_ptr(), stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.augment_batch(descs, src.data_ptr(), params, out, dst.data_ptr(), stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ctx.close()
    return dt * 1e6


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.cuda.set_device(0)
    print("C2 us/step", round(run(C.C2_AUG, steps), 1), flush=True)
    print("C2 + rotate [-15,15] us/step", round(run(dict(C.C2_AUG, angle=[-15, 15]), steps), 1), flush=True)
