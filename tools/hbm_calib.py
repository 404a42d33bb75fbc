"""Practical HBM rates on this GPU, back to back (torch's fill / copy kernels): python tools/hbm_calib.py.
Prints GB/s for a 402 MB fill (C5's image output), a 154 MB fill (C2's), and 200 MB -> 200 MB copies."""
import torch

torch.cuda.set_device(0)


def rate(fn, nbytes, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return nbytes / (ms * 1e-3) / 1e9, ms * 1e3


for mb in (154, 402):
    n = mb * (1 << 20) // 4
    a = torch.empty(n, dtype=torch.float32, device="cuda")
    g, us = rate(lambda: a.fill_(1.5), n * 4)
    print(f"fill {mb} MB: {g:7.0f} GB/s ({us:.1f} us)", flush=True)
    del a
for mb in (100, 200):
    n = mb * (1 << 20) // 4
    a = torch.empty(n, dtype=torch.float32, device="cuda")
    b = torch.empty(n, dtype=torch.float32, device="cuda")
    g, us = rate(lambda: b.copy_(a), 2 * n * 4)
    print(f"copy {mb} MB -> {mb} MB: {g:7.0f} GB/s (read + write, {us:.1f} us)", flush=True)
