"""Run glds_probe.hip: LDS-DMA dword / dwordx3 / dwordx4 placement and bounds (development only)."""
import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libglds_probe.so"))
src = (torch.arange(2048, dtype=torch.int32) % 251).to(torch.uint8).cuda()
host = src.cpu().numpy()
out = torch.zeros(256, dtype=torch.int32, device="cuda")
for size, base, nbytes, far in ((4, 1, 2048, 0), (4, 0, 192, 0), (4, 0, 2048, 1), (12, 0, 2048, 0), (12, 3, 2048, 0),
                                (12, 0, 12 * 63 + 6, 0), (16, 0, 2048, 0), (16, 5, 2048, 0)):
    L.launch(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()), nbytes, base, far, size)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint8)
    step = 3 if size == 4 else size
    exp = np.full(1024, 0xEF, np.uint8).reshape(256, 4)
    exp[:] = np.frombuffer(np.uint32(0xdeadbeef).tobytes(), np.uint8)
    exp = exp.reshape(-1)
    for l in range(64):
        o = base + step * l
        chunk = host[o:o + size].copy() if o + size <= nbytes and not (far and l == 5) else np.zeros(size, np.uint8)
        exp[l * size:(l + 1) * size] = chunk
    ok = np.array_equal(got, exp)
    print(f"size={size} base={base} nbytes={nbytes} far={far}: {'lane*size contiguous OK' if ok else 'MISMATCH'}")
    if not ok:
        print("  got[0:48]", got[:48].tolist())
        print("  exp[0:48]", exp[:48].tolist())
