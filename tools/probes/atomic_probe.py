"""Development: time device-scope work-counter atomics (tools/probes/atomic_probe.hip)."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "libatomic_probe.so"))
ctr = torch.zeros(64 * 1024, dtype=torch.int32, device="cuda")
out = torch.zeros(8192 + 768 * 16, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()


def run(grid, k, spread, spin, threads=448):
    ctr.zero_()
    L.ticket_launch(ctypes.c_void_p(ctr.data_ptr()), ctypes.c_void_p(out.data_ptr()), grid, threads, k, spread, spin,
                    ctypes.c_void_p(st.cuda_stream))


for grid, k, spread, spin in [(768, 1, 1, 0), (768, 4, 1, 0), (768, 4, 8, 0), (768, 4, 768, 0), (768, 16, 1, 0),
                              (768, 16, 8, 0), (768, 16, 768, 0), (768, 4, 1, 20), (768, 4, 8, 20), (768, 4, 768, 20)]:
    for _ in range(3):
        run(grid, k, spread, spin)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run(grid, k, spread, spin)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"grid {grid} tickets/wg {k:2d} counters {spread:3d} spin {spin:2d}: {us:7.2f} us/launch "
          f"({us / k:6.2f} us per ticket round)", flush=True)

# uniqueness: tickets of each counter must be a permutation of 0..n-1 (cross-XCD coherence)
for spread in (1, 8):
    run(768, 16, spread, 0)
    torch.cuda.synchronize()
    t = out[8192:8192 + 768 * 16].view(768, 16).cpu()
    ok = True
    for c in range(spread):
        v = t[[w for w in range(768) if w % spread == c]].flatten().sort().values
        ok &= bool((v == torch.arange(len(v), dtype=v.dtype)).all())
    print(f"counters {spread}: tickets unique and complete: {ok}")
