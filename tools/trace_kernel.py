"""Development: per-phase s_memtime stamps of the streaming kernel (C2), via AEON_HIP_TRACE_PTR.
Phases per iteration: 0 start, 1 after next-tile prep issued, 2 after compute, 3 after the counted
wait, 4 after the barrier; slot 7 of iteration 0 = kernel entry."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

tr = torch.zeros(8192 * 16 * 8, dtype=torch.int32, device="cuda")
os.environ["AEON_HIP_TRACE_PTR"] = str(tr.data_ptr())
import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

torch.cuda.set_device(0)
bench.run_device(A, C, torch, sys.argv[1] if len(sys.argv) > 1 else "C2", 256, 3, 1, 0, 1, 400, None)
torch.cuda.synchronize()
t = tr.cpu().numpy().view(np.uint32).reshape(8192, 16, 8).astype(np.int64)
used = np.nonzero(t[:, 0, 7])[0]
t = t[used]
t0 = t[:, 0, 7].min()
entry = t[:, 0, 7] - t0
print(f"workgroups {len(used)}; entry spread {entry.min()}..{entry.max()} ticks")
end = []
for w in range(len(t)):
    its = [i for i in range(16) if t[w, i, 0]]
    last = its[-1]
    end.append((t[w, last, 2] if t[w, last, 2] else t[w, last, 1]) - t0)
end = np.array(end)
print(f"workgroup end: min {end.min()} median {np.median(end):.0f} max {end.max()} ticks")
d = []
for w in range(len(t)):
    for i in range(16):
        r = t[w, i]
        if r[0] and r[3] and i + 1 < 16 and t[w, i + 1, 0]:
            d.append([r[1] - r[0], r[2] - r[1], r[3] - r[2], t[w, i + 1, 0] - r[3]])
d = np.array(d)
print("per full iteration (median ticks): prep %d  compute %d  wait %d  fix %d" % tuple(np.median(d, axis=0)))
print("prologue (entry -> first iteration start) median:", np.median(t[:, 0, 0] - t[:, 0, 7]))
life = end - entry
print("wave life median %d ticks; iterations per wave median %d" % (np.median(life), np.median([sum(1 for i in range(16) if t[w, i, 0]) for w in range(len(t))])))
