"""Development: per-phase s_memtime stamps of the record-resident contrast kernel (C3), via
AEON_HIP_TRACE_PTR.  Needs a trace build (the product library compiles the stamps out):
  tools/build_variants.sh trace=-DAEON_HIP_TRACE
  AEON_HIP_LIB=aeon_amd/variants/trace.so python tools/trace_records.py [real]
Layout [workgroup][step*8 + tile][32]: slots 0 tile top, 1 staging landed, 2 unpacked, 3 barrier passed,
4 next staging issued (lane 0 of wave 0); 16 + w = wave w done with the tile's rows; entry step*8+7:
0 record done, 1 sums barrier passed, 2 record table, 3 next record's tables; entry 63: s_memrealtime /
s_memtime at entry (0, 1) and exit (2, 3)."""
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

real = len(sys.argv) > 1 and sys.argv[1] == "real"
torch.cuda.set_device(0)
bench.run_device(A, C, torch, "C3", 1024, 1, 2, 0, 1, 600, None, real=real)
torch.cuda.synchronize()
t = tr.cpu().numpy().view(np.uint32)[:256 * 64 * 32].reshape(256, 64, 32).astype(np.int64)
used = np.nonzero(t[:, 63, 0])[0]
t = t[used]
nwg = len(t)
ent_rt, ent_mt, ext_rt, ext_mt = t[:, 63, 0], t[:, 63, 1], t[:, 63, 2], t[:, 63, 3]
tpu = np.median((ext_mt - ent_mt) / np.maximum((ext_rt - ent_rt) / 100.0, 1e-3))
print(f"{'real' if real else 'noise'} sources: workgroups {nwg}, s_memtime ticks/us {tpu:.0f}")
r0 = ent_rt.min()
print("entry us p0/p50/max %.2f %.2f %.2f; exit us p0/p50/p90/max %.2f %.2f %.2f %.2f" % (
    (ent_rt.min() - r0) / 100, np.median(ent_rt - r0) / 100, (ent_rt.max() - r0) / 100, (ext_rt.min() - r0) / 100,
    np.median(ext_rt - r0) / 100, np.percentile(ext_rt - r0, 90) / 100, (ext_rt.max() - r0) / 100))


def us(x):
    return x / tpu


nw = int(max(((t[:, :56, 16:32] > 0).any(axis=(0, 1))).nonzero()[0]) + 1)
print(f"waves stamped: {nw}")
print("per step k, tile t (median us over workgroups): wait unpack barrier issue | wave ends after the barrier: "
      "min med max (per-wave medians)")
for k in range(5):
    for tt in range(7):
        e = t[:, k * 8 + tt]
        if not e[:, 0].any():
            continue
        ok = e[:, 0] > 0
        e = e[ok]
        wend = e[:, 16:16 + nw] - e[:, 3:4]
        has1 = e[:, 1] > 0
        wait = np.where(has1, e[:, 1] - e[:, 0], 0)
        unp = np.where(has1, e[:, 2] - e[:, 1], 0)
        bar = e[:, 3] - np.where(has1, e[:, 2], e[:, 0])
        iss = e[:, 4] - e[:, 3]
        wm = np.median(wend, axis=0)
        print(f"  k{k} t{tt}: " + " ".join(f"{us(np.median(v)):6.2f}" for v in (wait, unp, bar, iss)) +
              " | " + " ".join(f"{us(v):5.2f}" for v in (wm.min(), np.median(wm), wm.max())) +
              "  [" + " ".join(f"{us(v):.1f}" for v in wm) + "]")
    e = t[:, k * 8:k * 8 + 7]
    if (e[:, :, 7] > 0).any():
        ok = e[:, :, 7] > 0
        print(f"  k{k} helper staging (median us): issue+taps {us(np.median((e[:, :, 5] - e[:, :, 3])[ok])):.2f}"
              f" wait {us(np.median((e[:, :, 6] - e[:, :, 5])[ok])):.2f} unpack {us(np.median((e[:, :, 7] - e[:, :, 6])[ok])):.2f}")
    e = t[:, k * 8 + 7]
    if e[:, 0].any():
        print(f"  k{k} end: sums+barrier {us(np.median(e[:, 1] - e[:, 0])):.2f} table {us(np.median(e[:, 2] - e[:, 1])):.2f}"
              f" next tables {us(np.median(e[:, 3] - e[:, 2])):.2f}")
steps = []
for k in range(5):
    a = t[:, k * 8, 3]
    b = t[:, k * 8 + 7, 3] if k < 4 else t[:, 63, 3]
    ok = (a > 0) & (b > 0)
    if ok.any():
        steps.append(us(np.median(b[ok] - a[ok])))
print("step durations (median us):", " ".join(f"{v:.1f}" for v in steps))
pro = us(np.median(t[:, 0, 3] - ent_mt))
hw = t[:, 62, 16:16 + nw]
simd = (hw >> 4) & 3
print("SIMD of each wave (workgroup 0):", simd[0].tolist(), " waves per SIMD:",
      [int((simd[0] == q).sum()) for q in range(4)])
# per tile: the last wave end of each SIMD after the barrier (median over workgroups and A-tiles)
ends = {q: [] for q in range(4)}
for k in range(4):
    for tt in range(7):
        e = t[:, k * 8 + tt]
        if not e[:, 0].any():
            continue
        w = e[:, 16:16 + nw] - e[:, 3:4]
        for q in range(4):
            m = np.where(simd == q, w, -1 << 40).max(axis=1)
            ends[q].extend(m.tolist())
print("per-tile last wave end after the barrier, by SIMD (median us): " +
      "  ".join(f"SIMD{q} {us(np.median(v)):.2f}" for q, v in ends.items() if v))
xcd = used % 8
print("exit us per XCD (median / max): " + "  ".join(
    f"{x}: {np.median(ext_rt[xcd == x] - r0) / 100:.1f}/{(ext_rt[xcd == x] - r0).max() / 100:.1f}" for x in range(8)))
print(f"prologue (entry -> first tile) {pro:.2f} us")
