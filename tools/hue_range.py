"""Exhaustive check behind the hue kernel's index arithmetic (augment_kernels.hip hue_apply_n):
over every BGR triple, OpenCV's RGB2HSV_b hue before the +180 wrap (h12) lies in [-30, 150], so the
wrapped H is in [0, 179] (its saturate_cast is a no-op) and equals min_u32(h12, h12 + 180).
python tools/hue_range.py  (tests/test_hue_range.py runs the same check)."""
import numpy as np


def check():
    i = np.arange(1, 256)
    hdiv = np.zeros(256, np.int64)
    hdiv[1:] = np.rint((180 << 12) / (6. * i)).astype(np.int64)
    lo, hi = 1 << 30, -(1 << 30)
    g, r = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    g, r = g.ravel(), r.ravel()
    for b in range(256):
        v = np.maximum(b, np.maximum(g, r))
        d = v - np.minimum(b, np.minimum(g, r))
        h = np.where(v == r, g - b, np.where(v == g, b - r + 2 * d, r - g + 4 * d))
        h12 = (h * hdiv[d] + (1 << 11)) >> 12
        wrapped = np.where(h12 < 0, h12 + 180, h12)
        via_min = np.minimum(h12.astype(np.uint32), (h12 + 180).astype(np.uint32)).astype(np.int64)
        assert np.array_equal(wrapped, via_min)
        lo, hi = min(lo, int(h12.min())), max(hi, int(h12.max()))
    return lo, hi


if __name__ == "__main__":
    print("h12 range", check())
