"""Development: per-phase s_memtime stamps of the band kernel (C2), via AEON_HIP_TRACE_PTR.
Needs a trace build (the product library compiles the stamps out):
  tools/build_variants.sh trace=-DAEON_HIP_TRACE
  AEON_HIP_LIB=aeon_amd/variants/trace.so python tools/trace_kernel.py C2
Layout [workgroup][iteration 0..15][slot 0..15]; slot 15 of iteration 0 / 1 = s_memrealtime
(chip-wide 100 MHz) at kernel entry / exit, slot 14 of iteration 0 = s_memtime at entry.  Single-buffered phases: 0 start, 1 info, 2 DMA
issued, 3 tap tables, 4 loads landed, 5 unpacked, 6 barrier, 7 computed, 8 end barrier.
Double-buffered: 0 start, 1 next prep issued, 2 computed, 3 counted wait, 4 unpacked, 5 barrier."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

tr = torch.zeros(8192 * 16 * 16, dtype=torch.int32, device="cuda")
os.environ["AEON_HIP_TRACE_PTR"] = str(tr.data_ptr())
import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402

torch.cuda.set_device(0)
# TRACE_ISOLATED=1: the traced launch alone (one timed step after a synchronize), else the last of three
# back-to-back launches
iso = os.environ.get("TRACE_ISOLATED") == "1"
bench.run_device(A, C, torch, sys.argv[1] if len(sys.argv) > 1 else "C2", 256, 1 if iso else 3, 2 if iso else 1, 0, 1, 400, None)
torch.cuda.synchronize()
t = tr.cpu().numpy().view(np.uint32).reshape(8192, 16, 16).astype(np.int64)
used = np.nonzero(t[:, 0, 15])[0]
t = t[used]
print(f"workgroups {len(used)}")

# per-iteration phase durations (s_memtime ticks; per-XCD clocks, so only differences)
nph = 9
d = []
for w in range(len(t)):
    for i in range(15):
        r = t[w, i, :nph]
        if r[0] and r[nph - 1]:
            d.append(np.diff(r))
d = np.array(d)
names = ["info", "dma-issue", "tables", "wait", "unpack", "barrier", "compute", "end-barrier"]
print("per tile, median ticks: " + "  ".join(f"{n} {v:.0f}" for n, v in zip(names, np.median(d, axis=0))))
print("per tile, mean ticks:   " + "  ".join(f"{n} {v:.0f}" for n, v in zip(names, np.mean(d, axis=0))))
its = np.array([sum(1 for i in range(15) if t[w, i, 0]) for w in range(len(t))])
print("tiles per workgroup:", {int(k): int((its == k).sum()) for k in np.unique(its)})

# global timeline from s_memrealtime
ent = t[:, 0, 15]
ext = t[:, 1, 15]
ok = ext > 0
r0 = ent[ok].min()
ent_us = (ent[ok] - r0) / 100.0
ext_us = (ext[ok] - r0) / 100.0
life_ticks = np.array([max(t[w, i, :nph].max() for i in range(15) if t[w, i, 0]) - t[w, 0, 0] for w in range(len(t))])[ok]
life_us = ext_us - ent_us
print("realtime: entry us p0/p50/p90/max %.2f %.2f %.2f %.2f" % (ent_us.min(), np.median(ent_us), np.percentile(ent_us, 90), ent_us.max()))
print("realtime: exit  us p10/p50/p90/max %.2f %.2f %.2f %.2f" % (np.percentile(ext_us, 10), np.median(ext_us), np.percentile(ext_us, 90), ext_us.max()))
print("s_memtime ticks per us (median over workgroups): %.0f" % np.median(life_ticks / np.maximum(life_us, 1e-3)))
wid = used[ok]
print("entry us p50 by blockIdx eighth: " + " ".join("%.2f" % np.median(ent_us[(wid * 8 // 768) == k]) for k in range(8)))
print("entries per us:", [int(((ent_us >= b) & (ent_us < b + 1)).sum()) for b in range(int(np.ceil(ent_us.max())) + 1)])
for xcd in range(8):
    s = wid % 8 == xcd
    print("realtime xcd %d: exit p10/p50/p90/max %.2f %.2f %.2f %.2f" % (xcd, np.percentile(ext_us[s], 10), np.median(ext_us[s]),
                                                                   np.percentile(ext_us[s], 90), ext_us[s].max()))

# the ramp: entry -> first tile's loop start (prologue: LUT + first jobs) -> first compute (first stores)
tpu = np.median(life_ticks / np.maximum(life_us, 1e-3))
pro = (t[ok, 0, 0] - t[ok, 0, 14]) / tpu
first = (t[ok, 0, 6] - t[ok, 0, 14]) / tpu
print("prologue us p10/p50/p90 %.2f %.2f %.2f; entry -> first compute us p10/p50/p90 %.2f %.2f %.2f" % (
    np.percentile(pro, 10), np.median(pro), np.percentile(pro, 90), np.percentile(first, 10), np.median(first),
    np.percentile(first, 90)))
fc_rt = ent_us + first
print("first compute (realtime us from first entry) p10/p50/p90/max %.2f %.2f %.2f %.2f" % (
    np.percentile(fc_rt, 10), np.median(fc_rt), np.percentile(fc_rt, 90), fc_rt.max()))
# workgroups computing (phase 6 -> 7) over time, 1 us bins
spans = []
for w in np.nonzero(ok)[0]:
    for i in range(15):
        if t[w, i, 0] and t[w, i, 7]:
            spans.append(((t[w, i, 6] - t[w, 0, 14]) / tpu + ent_us[np.searchsorted(np.nonzero(ok)[0], w)],
                          (t[w, i, 7] - t[w, 0, 14]) / tpu + ent_us[np.searchsorted(np.nonzero(ok)[0], w)]))
spans = np.array(spans)
end = int(np.ceil(ext_us.max()))
busy = [int(((spans[:, 0] < b + 1) & (spans[:, 1] > b)).sum()) for b in range(end)]
print("workgroups in compute per us:", busy)

# prologue parts (slots 10..13 of iteration 0: jobs issued, vmcnt(0) done, barrier done, info derived)
parts = {"issue": (14, 10), "wait": (10, 11), "barrier": (11, 12), "info": (12, 13), "to-loop": (13, 0)}
print("prologue parts us p50/p90: " + "  ".join(
    f"{k} {np.median((t[ok, 0, b] - t[ok, 0, a]) / tpu):.2f}/{np.percentile((t[ok, 0, b] - t[ok, 0, a]) / tpu, 90):.2f}"
    for k, (a, b) in parts.items()))
