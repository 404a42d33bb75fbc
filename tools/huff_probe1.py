import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
import aeon_amd as A
FX = np.load("tests/golden/jpeg_fixtures.npz")
for name in sys.argv[1:]:
    f = FX[name + ".jpg"].tobytes()
    w, h, _ = A.jpeg_info(f)
    ctx = A.Context(0)
    dst = torch.empty(w * h * 3 + 16, dtype=torch.uint8, device="cuda")
    d = (A.ImgDesc * 1)(A.ImgDesc(offset=0, width=w, height=h, stride=w * 3, channels=3))
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(2):
        print("== call", name, flush=True)
        ctx.decode_jpeg_batch([f], d, dst.data_ptr(), s)
        ctx.synchronize(s)
    ctx.close()
