"""Run lds_unaligned.hip: are byte-unaligned ds_read_b32 / ds_read_b64 exact? (development only)"""
import ctypes
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "liblds_unaligned.so"))
out = torch.zeros(64 * 3, dtype=torch.int32, device="cuda")
for stride in (3, 6, 12):
    L.launch(ctypes.c_void_p(out.data_ptr()), stride)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32).reshape(64, 3)
    bad = 0
    for l in range(64):
        a = stride * l + 1
        b = [(a + k) & 0xff for k in range(8)]
        e32 = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24
        e64y = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24
        if got[l, 0] != e32 or got[l, 1] != e32 or got[l, 2] != e64y:
            bad += 1
            if bad < 3:
                print("  lane", l, [hex(x) for x in got[l]], hex(e32), hex(e64y))
    print(f"stride {stride}: {'exact' if not bad else f'{bad} lanes differ'}")
