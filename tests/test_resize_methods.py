"""CPU: the oracle's cv::resize restatements for CUBIC, AREA and LANCZOS4 (aeon's interpolation_method
map, /root/reference/src/image.cpp:30-36, used by image::resize :93-106 and resize_short :118-127).

PARITY UNPINNED: aeon's own tests hold no output of these methods and OpenCV is absent here, so the
restatement (oracle/aeon_oracle.cpp resize_cv, from OpenCV 2.4.9 imgwarp.cpp) is checked for the
properties the published algorithm has -- identity at equal size, constants kept, an ideal
double-precision evaluation of the same filter within its fixed-point rounding, exact box means for
integer INTER_AREA factors, the area-mode bilinear emulation for upscales -- not against reference
output.  The GPU is compared with this restatement bit for bit in tests/test_hip_parity.py.
"""
import numpy as np
import pytest

import oracle as O


def _img(h, w, seed, cn=3):
    return np.random.default_rng(seed).integers(0, 256, (h, w, cn), dtype=np.uint8)


def _cubic(x):
    A = -0.75
    return np.array([((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A,
                     ((A + 2) * x - (A + 3)) * x * x + 1,
                     ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1,
                     0.0])


def _ideal(src, dw, dh, method):
    """The same separable filter in double precision (no fixed point), taps clamped at the edges."""
    h, w, cn = src.shape
    k = 4 if method == "CUBIC" else 8
    k2 = k // 2

    def taps(n_src, n_dst):
        sc = n_src / n_dst
        out = []
        for d in range(n_dst):
            f = (d + 0.5) * sc - 0.5
            s = int(np.floor(f))
            f -= s
            if s < 0:
                f, s = 0.0, 0
            if s >= n_src - 1:
                f, s = 0.0, n_src - 1
            if method == "CUBIC":
                c = _cubic(f)
                c[3] = 1 - c[:3].sum()
            else:
                c = O.lanczos4_coeffs(f).astype(np.float64)
            idx = np.clip(s - k2 + 1 + np.arange(k), 0, n_src - 1)
            out.append((idx, c))
        return out

    def rows_taps(n_src, n_dst):  # y: raw sy, rows clipped
        sc = n_src / n_dst
        out = []
        for d in range(n_dst):
            f = (d + 0.5) * sc - 0.5
            s = int(np.floor(f))
            f -= s
            c = _cubic(f) if method == "CUBIC" else O.lanczos4_coeffs(f).astype(np.float64)
            if method == "CUBIC":
                c[3] = 1 - c[:3].sum()
            out.append((np.clip(s - k2 + 1 + np.arange(k), 0, n_src - 1), c))
        return out

    xs, ys = taps(w, dw), rows_taps(h, dh)
    tmp = np.stack([(src[:, i, :].astype(np.float64) * c[None, :, None]).sum(1) for i, c in xs], 1)
    out = np.stack([(tmp[i, :, :] * c[:, None, None]).sum(0) for i, c in ys], 0)
    return np.clip(np.rint(out), 0, 255)


@pytest.mark.parametrize("method", ["CUBIC", "AREA", "LANCZOS4"])
def test_identity_and_constants(method):
    im = _img(37, 53, 1)
    assert np.array_equal(O.resize(im, 53, 37, method), im)
    c = np.full((40, 60, 3), 77, np.uint8)
    for dw, dh in ((23, 17), (131, 97), (60, 13), (7, 40)):
        assert np.unique(O.resize(c, dw, dh, method)).tolist() == [77], (method, dw, dh)


@pytest.mark.parametrize("method", ["CUBIC", "LANCZOS4"])
@pytest.mark.parametrize("size", [(224, 224), (100, 61), (300, 280), (31, 47)])
def test_generic_filters_match_ideal_filter(method, size):
    """11-bit coefficients and the SSE2 / FixedPtCast vertical pass stay within 2 of the ideal
    double-precision filter with the same taps and edge clamps."""
    src = _img(180, 200, 5)
    got = O.resize(src, size[0], size[1], method).astype(np.int32)
    want = _ideal(src, size[0], size[1], method)
    assert np.abs(got - want).max() <= 2


def test_area_integer_factors_are_box_means():
    src = _img(96, 120, 7)
    for f in (2, 3, 4):
        got = O.resize(src, 120 // f, 96 // f, "AREA").astype(np.float64)
        box = src.reshape(96 // f, f, 120 // f, f, 3).astype(np.float64).mean((1, 3))
        assert np.abs(got - box).max() <= 0.5 + 1e-9, f  # rounding of the mean only
        if f == 2:  # the 2x2 fast mode: (a + b + c + d + 2) >> 2
            s = src.reshape(48, 2, 60, 2, 3).astype(np.int32).sum((1, 3))
            assert np.array_equal(got.astype(np.int32), (s + 2) >> 2)


def test_area_generic_is_the_area_average():
    """Non-integer downscale: each output is the area-weighted mean of the source cells it covers."""
    src = _img(100, 130, 9)
    dw, dh = 57, 43
    got = O.resize(src, dw, dh, "AREA").astype(np.float64)
    sx, sy = 130 / dw, 100 / dh

    def weights(n_src, n_dst, sc):
        m = np.zeros((n_dst, n_src))
        for d in range(n_dst):
            a, b = d * sc, (d + 1) * sc
            for s in range(int(np.floor(a)), min(int(np.ceil(b)), n_src)):
                m[d, s] = max(0.0, min(b, s + 1) - max(a, s))
        return m / m.sum(1, keepdims=True)

    wx, wy = weights(130, dw, sx), weights(100, dh, sy)
    ideal = np.einsum("ys,xt,stc->yxc", wy, wx, src.astype(np.float64))
    assert np.abs(got - ideal).max() <= 1.0


def test_area_upscale_is_area_mode_bilinear():
    """INTER_AREA with an upscaled axis: bilinear taps from the area-mode coefficients -- a source
    pixel's value repeats over its cell, blending only across the cell boundaries."""
    src = _img(10, 12, 11)
    got = O.resize(src, 36, 30, "AREA")  # 3x in both axes: every output lies inside one cell
    assert np.array_equal(got, np.repeat(np.repeat(src, 3, 0), 3, 1))
    got2 = O.resize(src, 30, 10, "AREA")  # 2.5x in x only
    assert got2.shape == (10, 30, 3)
    assert np.array_equal(got2[:, 0], src[:, 0]) and np.array_equal(got2[:, -1], src[:, -1])
