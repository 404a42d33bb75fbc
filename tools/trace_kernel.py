"""Development: per-phase s_memtime stamps of the streaming kernel (C2), via AEON_HIP_TRACE_PTR.
Phases per iteration, double-buffered: 0 start, 1 after next-tile prep issued, 2 after compute, 3
after the counted wait, 4 after the unpack, 5 after the barrier; single-buffered: 0 start, 1 prep
issued, 2 loads landed, 3 unpacked, 4 barrier, 5 computed.  Slot 7 of iteration 0 = kernel entry
(s_memrealtime), slot 7 of iteration 1 = exit."""
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
    end.append(max(t[w, last, :7]) - t0)
end = np.array(end)
print(f"workgroup end: min {end.min()} median {np.median(end):.0f} max {end.max()} ticks")
d = []
for w in range(len(t)):
    for i in range(16):
        r = t[w, i]
        if r[0] and r[5]:
            d.append([r[1] - r[0], r[2] - r[1], r[3] - r[2], r[4] - r[3], r[5] - r[4]])
d = np.array(d)
print("per full iteration (median ticks) phase deltas 1..5: %d %d %d %d %d" % tuple(np.median(d, axis=0)))
print("per full iteration (mean ticks)   phase deltas 1..5: %d %d %d %d %d" % tuple(np.mean(d, axis=0)))
print("prologue (entry -> first iteration start) median:", np.median(t[:, 0, 0] - t[:, 0, 7]))
life = end - entry
print("wave life median %d ticks; iterations per wave median %d" % (np.median(life), np.median([sum(1 for i in range(16) if t[w, i, 0]) for w in range(len(t))])))

# per-XCD view (workgroup i runs on XCD i % 8; each XCD has its own clock): entry and exit times
# relative to the XCD's first entry
ids = used
for xcd in range(8):
    sel = [k for k, w in enumerate(ids) if w % 8 == xcd]
    if not sel:
        continue
    e = t[sel, 0, 7]
    x0 = e.min()
    ends = []
    for k in sel:
        its = [i for i in range(16) if t[k, i, 0]]
        last = its[-1]
        ends.append(max(t[k, last, :7]) - x0)
    ent = e - x0
    print(f"xcd {xcd}: {len(sel)} wgs, entry p50 {np.median(ent):.0f} p90 {np.percentile(ent, 90):.0f} max {ent.max()}, "
          f"end p10 {np.percentile(ends, 10):.0f} p50 {np.median(ends):.0f} max {max(ends)}")

# global timeline from s_memrealtime (100 MHz, chip-wide): slot [wg, 0, 7] entry, [wg, 1, 7] exit
ent = t[:, 0, 7].astype(np.int64)
ext = t[:, 1, 7].astype(np.int64)
ok = ext > 0
r0 = ent[ok].min()
ent_us = (ent[ok] - r0) / 100.0
ext_us = (ext[ok] - r0) / 100.0
print("realtime: entry us p0/p50/p90/max %.2f %.2f %.2f %.2f" % (ent_us.min(), np.median(ent_us), np.percentile(ent_us, 90), ent_us.max()))
print("realtime: exit  us p10/p50/p90/max %.2f %.2f %.2f %.2f" % (np.percentile(ext_us, 10), np.median(ext_us), np.percentile(ext_us, 90), ext_us.max()))
print("realtime: workgroup life us p50 %.2f" % np.median(ext_us - ent_us))
nits = np.array([sum(1 for i in range(16) if t[w, i, 0]) for w in range(len(t))])[ok]
for k in sorted(set(nits.tolist())):
    s = nits == k
    print("realtime: %d-tile workgroups: %d, entry p50 %.2f, exit p10/p50/max %.2f %.2f %.2f us"
          % (k, s.sum(), np.median(ent_us[s]), np.percentile(ext_us[s], 10), np.median(ext_us[s]), ext_us[s].max()))
wid = used[ok]
for xcd in range(8):
    s = wid % 8 == xcd
    print("realtime xcd %d: exit p10/p50/p90/max %.2f %.2f %.2f %.2f" % (xcd, np.percentile(ext_us[s], 10), np.median(ext_us[s]),
                                                                   np.percentile(ext_us[s], 90), ext_us[s].max()))
for q in range(0, len(wid), 96):
    s = (wid >= q) & (wid < q + 96)
    print("realtime wg %4d..%4d: entry p50 %.2f exit p10/p50/max %.2f %.2f %.2f" % (q, q + 95, np.median(ent_us[s]), np.percentile(ext_us[s], 10),
                                                                             np.median(ext_us[s]), ext_us[s].max()))
