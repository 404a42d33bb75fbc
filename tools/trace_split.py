"""Development: per-phase s_memtime stamps of augment_split (C2), via AEON_HIP_TRACE_PTR.
Needs a trace build (the product library compiles the stamps out):
  tools/build_variants.sh trace=-DAEON_HIP_TRACE
  AEON_HIP_LIB=aeon_amd/variants/trace.so python tools/trace_split.py
Layout [workgroup][tile k < 15][slot]: slots 0-4 by the last wave (staging only), 8-12 by wave 0 (compute):
iteration start, tile k + 2 issued, tile k computed, tile k + 1's loads landed, unpacked; tile 15: slot 13
s_memtime at entry, 14 s_memrealtime at entry, 15 s_memrealtime at exit."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

tr = torch.zeros(4096 * 16 * 16, dtype=torch.int32, device="cuda")
os.environ["AEON_HIP_TRACE_PTR"] = str(tr.data_ptr())
import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

torch.cuda.set_device(0)
bench.run_device(A, C, torch, sys.argv[1] if len(sys.argv) > 1 else "C2", 256, 3, 1, 0, 1, 400, None, 0)
torch.cuda.synchronize()
t = tr.cpu().numpy().view(np.uint32).reshape(4096, 16, 16).astype(np.int64)
used = np.nonzero(t[:, 15, 14])[0]
t = t[used]
nwg = len(used)
print(f"workgroups {nwg}")
ent_rt = t[:, 15, 14]
ext_rt = t[:, 15, 15]
ent_mt = t[:, 15, 13]
# ticks per us from each workgroup's life: helper exit realtime vs its last s_memtime stamp is not exact;
# use the compute stamps' span against the realtime span instead (s_memtime ~ 100 MHz * k)
K = np.array([sum(1 for k in range(15) if t[w, k, 8]) for w in range(nwg)])
last = np.array([t[w, K[w] - 1, 10] for w in range(nwg)])
life_rt_us = (ext_rt - ent_rt) / 100.0
tpu = np.median((last - ent_mt) / np.maximum(life_rt_us, 1e-3))
print(f"tiles per workgroup {dict(zip(*np.unique(K, return_counts=True)))}; s_memtime ticks/us ~{tpu:.0f}")
us = lambda x: x / tpu  # noqa: E731
r0 = ent_rt.min()
print("entry us p50/max %.2f %.2f; helper exit us p10/p50/p90/max %.2f %.2f %.2f %.2f" % (
    np.median((ent_rt - r0) / 100), (ent_rt - r0).max() / 100, *np.percentile((ext_rt - r0) / 100, [10, 50, 90, 100])))
first = us(t[:, 0, 8] - ent_mt)
print("entry -> tile 0 compute start us p10/p50/p90 %.2f %.2f %.2f" % tuple(np.percentile(first, [10, 50, 90])))
rows = []
for k in range(int(K.max())):
    m = K > k
    d = lambda a, b: us(np.where((t[m, k, a] > 0) & (t[m, k, b] > 0), t[m, k, b] - t[m, k, a], 0))  # noqa: E731
    nxt = t[m, k + 1, 8] if k + 1 < 15 else 0 * t[m, k, 8]
    bar = us(np.where((nxt > 0) & (t[m, k, 12] > 0), nxt - t[m, k, 12], 0))
    rows.append((k, np.median(d(8, 9)), np.median(d(9, 10)), np.median(d(10, 11)), np.median(d(11, 12)), np.median(bar),
                 np.median(d(0, 1)), np.median(d(2, 3)), np.median(d(3, 4))))
print("tile  issue  compute  wait  unpack  barrier | staging-wave: issue  wait  unpack   (us, medians; wave 0 / last wave)")
for r in rows:
    print("%3d   %5.2f  %6.2f  %5.2f  %5.2f  %6.2f  |              %5.2f %5.2f %5.2f" % r)
for xcd in range(8):
    s = (used % 8) == xcd
    print("xcd %d: exit us p50/max %.2f %.2f" % (xcd, np.median((ext_rt[s] - r0) / 100), (ext_rt[s] - r0).max() / 100))
