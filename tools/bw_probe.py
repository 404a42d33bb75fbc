"""Measure achievable HBM rates for write-only and copy streams (the ceiling for this stage)."""
import torch

torch.cuda.set_device(0)
n = 154 * 1024 * 1024 // 4
x = torch.empty(n, dtype=torch.float32, device="cuda")
y = torch.empty(n, dtype=torch.float32, device="cuda")
big = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(4)]


def t(fn, reps=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


i = [0]


def fill():
    big[i[0] % 4].fill_(1.0)
    i[0] += 1


dt = t(fill)
print(f"fill  154MB: {dt*1e6:.1f} us  {n*4/dt/1e9:.0f} GB/s (write)")
dt = t(lambda: y.copy_(x))
print(f"copy  154MB: {dt*1e6:.1f} us  {2*n*4/dt/1e9:.0f} GB/s (read+write)")
dt = t(lambda: x.sum())
print(f"sum   154MB: {dt*1e6:.1f} us  {n*4/dt/1e9:.0f} GB/s (read)")
