"""aeon's own known-answer tests for the host geometry of make_params and for the loader,
restated against BOTH the product (aeon_amd, through the C ABI) and the CPU oracle.

Each test names the reference test it restates (test/test_util.cpp, test/test_image.cpp);
the expected values are the reference's literals.  The loader KATs (BGR->RGB / layout,
standardize) run the product on the GPU (-m gpu) and the oracle on the CPU.
"""
import numpy as np
import pytest

import aeon_amd as A


def _impls(oracle):
    """(name, unbiased_round, calculate_scale, cropbox_max_proportional) for product and oracle."""
    return [("aeon_amd", A.unbiased_round, A.calculate_scale, A.cropbox_max_proportional),
            ("oracle", oracle.unbiased_round, oracle.calculate_scale, oracle.cropbox_max_proportional)]


# test/test_util.cpp:397-412 TEST(util, unbiased_round)
UNBIASED = [(1.5, 2), (2.5, 2), (-0.5, 0), (0.5, 0), (622.5, 622), (621.5, 622), (1.1, 1), (2.1, 2),
            (900.9, 901), (-1.1, -1), (-2.1, -2), (-2.5, -2), (-1.5, -2)]


def test_kat_unbiased_round(oracle):
    for name, ur, _, _ in _impls(oracle):
        for x, want in UNBIASED:
            assert ur(x) == want, (name, x)


# test/test_image.cpp:831-872 TEST(image, cropbox_max_proportional)
CROPBOX = [((100, 50), (200, 100), (100, 50)), ((100, 50), (50, 25), (100, 50)),
           ((100, 50), (200, 50), (100, 25)), ((100, 50), (50, 100), (25, 50)),
           ((100, 50), (10, 10), (50, 50))]


def test_kat_cropbox_max_proportional(oracle):
    for name, _, _, cmp_ in _impls(oracle):
        for (iw, ih), (ow, oh), want in CROPBOX:
            assert cmp_(iw, ih, ow, oh) == want, (name, (iw, ih), (ow, oh))


def test_kat_calculate_scale(oracle):
    """test/test_image.cpp:874-886 TEST(image, calculate_scale): 500x375 into 800x800 -> 1.6,
    unbiased_round(500*1.6) x unbiased_round(375*1.6) = 800 x 600."""
    for name, ur, cs, _ in _impls(oracle):
        s = cs(500, 375, 800, 800)
        assert np.float32(s) == np.float32(1.6), name
        f32 = np.float32
        assert (ur(float(f32(500) * f32(s))), ur(float(f32(375) * f32(s)))) == (800, 600), name


def test_kat_area_scale(oracle):
    """test/test_image.cpp:1006-1047 TEST(image, area_scale): do_area_scale keeps the aspect
    ratio and cuts the area ratio down to what the image allows, both within 2e-4, through the
    product's and the oracle's make_params."""
    eps = 0.0002
    for w, h in ((40000, 20000), (30000, 30000), (20000, 40000)):
        src_area = np.float32(w * h)
        for area_ratio in (1.0, 0.8, 0.6, 0.4, 0.2, 0.07):
            for ar in (2 / 3, 9 / 16, 3 / 4, 1.0, 4 / 3, 16 / 9, 3 / 2):
                ar32, ratio32 = np.float32(ar), np.float32(area_ratio)
                bound = min(np.float32(w) / np.float32(h) / ar32, np.float32(h) / np.float32(w) * ar32)
                new_ratio = np.float32(src_area * min(ratio32, bound)) / src_area
                aug = {"type": "image", "flip_enable": False, "do_area_scale": True,
                       "scale": [float(ratio32)] * 2, "horizontal_distortion": [float(ar32)] * 2}
                prod = A.ParamFactory(aug).make_params(np.array([1], np.uint32), w, h, 256, 128)
                orc = oracle.Factory(oracle.aug_config(do_area_scale=1, scale_min=ratio32, scale_max=ratio32,
                                                       hdist_min=ar32, hdist_max=ar32)).make_params(
                    np.array([1], np.uint32), w, h, 256, 128)
                for name, p in (("aeon_amd", prod), ("oracle", orc)):
                    assert abs(ar - p.crop_w / p.crop_h) < eps, (name, w, h, area_ratio, ar)
                    assert abs(new_ratio - p.crop_w * p.crop_h / float(src_area)) < eps, (name, w, h, area_ratio, ar)
                assert (prod.crop_x, prod.crop_y, prod.crop_w, prod.crop_h) == \
                       (orc.crop_x, orc.crop_y, orc.crop_w, orc.crop_h)


def _indexed(rows, cols):
    """generate_indexed_image (test/test_image.cpp:42-57): b = col, g = row, r = 0."""
    img = np.zeros((rows, cols, 3), np.uint8)
    img[:, :, 0] = (np.arange(cols) % 256).astype(np.uint8)[None, :]
    img[:, :, 1] = (np.arange(rows) % 256).astype(np.uint8)[:, None]
    return img


def _bgr_to_rgb_expect(rows, cols, channel_major):
    """test/test_image.cpp:262-336: after bgr_to_rgb the planes/pixels are (0, row, col)."""
    rr, cc = np.meshgrid(np.arange(rows), np.arange(cols), indexing="ij")
    planes = np.stack([np.zeros_like(rr), rr, cc]).astype(np.uint8)
    return planes if channel_major else planes.transpose(1, 2, 0)


@pytest.mark.parametrize("channel_major", [False, True])
def test_kat_bgr_to_rgb_oracle(oracle, channel_major):
    """TEST(image, bgr_to_rgb[_channel_major]) (test/test_image.cpp:338-357), 10 x 20 uint8."""
    lc = oracle.load_config(3, channel_major, True, "uint8")
    out = oracle.load_image(_indexed(20, 10), lc)
    assert np.array_equal(out, _bgr_to_rgb_expect(20, 10, channel_major))


def _standardize_expect(img, mean, std):
    x = img.astype(np.float64) / 255.
    return np.stack([(x[..., c] - mean[c]) / (std[c] if std[c] else 1) for c in range(3)], axis=-1)


STD_MEAN = (0.5, 0.5, 0.0)
STD_DEV = (0.28980498288430989, 0.28980498288430989, 0.0)


def test_kat_standardize_oracle(oracle):
    """TEST(image, standardize) (test/test_image.cpp:379-429): HWC float, stddev 0 = no scaling,
    |err| <= 1e-5."""
    img = _indexed(256, 256)
    out = oracle.load_image(img, oracle.load_config(3, False, False, "float32", STD_MEAN, STD_DEV))
    assert np.abs(out - _standardize_expect(img, STD_MEAN, STD_DEV)).max() <= 1e-5


def _identity_params(w, h):
    return A.aug_params(crop_x=0, crop_y=0, crop_w=w, crop_h=h, out_w=w, out_h=h)


@pytest.mark.gpu
@pytest.mark.parametrize("channel_major", [False, True])
@pytest.mark.parametrize("fixed_aspect_ratio", [False, True])
def test_kat_bgr_to_rgb_gpu(channel_major, fixed_aspect_ratio):
    """TEST(image, bgr_to_rgb[_channel_major][_fixed_aspect_ratio]) (test/test_image.cpp:338-377):
    two 10 x 20 indexed records through the HIP loader (uint8, the config's default type)."""
    from tests import helpers as H
    ctx = A.Context(0)
    imgs = [_indexed(20, 10)] * 2
    out = A.out_desc(channels=3, channel_major=channel_major, bgr_to_rgb=True, dtype="uint8",
                     item_stride=10 * 20 * 3, fixed_aspect_ratio=fixed_aspect_ratio, canvas=(10, 20))
    params = [_identity_params(10, 20)] * 2
    res = H.hip_canvases(ctx, imgs, params, out) if fixed_aspect_ratio else H.hip_records(ctx, imgs, params, out)
    for r in res:
        assert np.array_equal(r, _bgr_to_rgb_expect(20, 10, channel_major))
    ctx.close()


@pytest.mark.gpu
def test_kat_standardize_gpu():
    """TEST(image, standardize) (test/test_image.cpp:379-429) through the HIP loader."""
    from tests import helpers as H
    ctx = A.Context(0)
    img = _indexed(256, 256)
    out = A.out_desc(channels=3, channel_major=False, dtype="float32", mean=STD_MEAN, stddev=STD_DEV,
                     item_stride=256 * 256 * 3 * 4)
    (res,) = H.hip_records(ctx, [img], [_identity_params(256, 256)], out)
    assert np.abs(res - _standardize_expect(img, STD_MEAN, STD_DEV)).max() <= 1e-5
    ctx.close()
