"""C5 kernel times: image (bilinear -> 512x512x3 f32 CHW) and pixel mask (nearest -> 512x512 u8)
launches timed separately (development tool)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    ctx = A.Context(0)
    batch, (w, h) = 128, (640, 480)
    img = torch.randint(0, 256, (batch * w * h * 3,), dtype=torch.uint8, device="cuda")
    msk = torch.randint(0, 21, (batch * w * h,), dtype=torch.uint8, device="cuda")
    idesc = (A.ImgDesc * batch)(*[A.ImgDesc(offset=i * w * h * 3, width=w, height=h, stride=w * 3, channels=3)
                                  for i in range(batch)])
    mdesc = (A.ImgDesc * batch)(*[A.ImgDesc(offset=i * w * h, width=w, height=h, stride=w, channels=1)
                                  for i in range(batch)])
    iout, mout = C.out_desc_for(C.IMAGE_512, C.C5_AUG), C.out_desc_for(C.MASK_512, C.C5_AUG)
    idst = torch.empty(batch * iout.item_stride, dtype=torch.uint8, device="cuda")
    mdst = torch.empty(batch * mout.item_stride, dtype=torch.uint8, device="cuda")
    f = A.ParamFactory(C.C5_AUG)
    st = A.seed_slots(1, batch)
    params = (A.AugParams * batch)(*[f.make_params(st[i:i + 1], w, h, 512, 512) for i in range(batch)])
    for name, fn, d, src, o, dst in (("image", ctx.augment_batch, idesc, img, iout, idst),
                                     ("mask", ctx.mask_batch, mdesc, msk, mout, mdst)):
        for _ in range(3):
            fn(d, src.data_ptr(), params, o, dst.data_ptr())
        torch.cuda.synchronize()
        ctx.kernel_times()
        ctx.set_timing(1)
        for _ in range(20):
            fn(d, src.data_ptr(), params, o, dst.data_ptr())
        torch.cuda.synchronize()
        ms, by, n = ctx.kernel_times()["augment"]
        ctx.set_timing(0)
        print(f"{name:6s} {ms / n * 1e3:.1f} us/launch  {by / n / 1e6:.1f} MB algorithmic  {by / ms / 1e6:.0f} GB/s", flush=True)
    ctx.close()
