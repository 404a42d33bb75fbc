"""Does a dword-unaligned raw_buffer_load_b128 return the bytes at its exact byte offset?"""
import ctypes
import os

import numpy as np
import torch

L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprobe.so"))
src = torch.arange(256, dtype=torch.int32).to(torch.uint8).cuda()
out = torch.zeros(64 * 16, dtype=torch.uint8, device="cuda")
L.probe_unaligned(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(out.data_ptr()), 256,
                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
got = out.cpu().numpy().reshape(64, 16)
exp = np.stack([np.arange(i, i + 16) % 256 for i in range(64)]).astype(np.uint8)
bad = [i for i in range(64) if not np.array_equal(got[i], exp[i])]
print("unaligned b128 exact:", not bad, "bad offsets:", bad[:8], "e.g. offset 1 ->", got[1][:8].tolist())
