"""GPU parity of the CUBIC / AREA / LANCZOS4 resizes (aeon's interpolation_method map,
/root/reference/src/image.cpp:30-36; image::resize :93-106 and resize_short :118-127) against the
oracle's cv::resize restatement (oracle/aeon_oracle.cpp resize_cv), bit for bit.

PARITY UNPINNED: aeon's tests hold no output of these methods and OpenCV is absent here; the
oracle's restatement of OpenCV 2.4.9 is itself checked only for the published algorithm's
properties (tests/test_resize_methods.py).  What these tests pin is that the HIP path
(resize_kernels.hip pre-pass + the tile kernel's copy pass) computes exactly that restatement.
"""
import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu

METHODS = {"CUBIC": A.INTERP_CUBIC, "AREA": A.INTERP_AREA, "LANCZOS4": A.INTERP_LANCZOS4}


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = A.Context(0)
    yield c
    c.close()


def _assert_same(hip, ref, what):
    assert len(hip) == len(ref)
    for i, (a, b) in enumerate(zip(hip, ref)):
        assert a.shape == b.shape, (what, i, a.shape, b.shape)
        if not np.array_equal(a, b):
            bad = np.argwhere(a != b)
            raise AssertionError(f"{what}: record {i}: {len(bad)} mismatches, first at {bad[0]}: "
                                 f"hip={a[tuple(bad[0])]} ref={b[tuple(bad[0])]}")


F32 = dict(channels=3, channel_major=True, bgr_to_rgb=True, dtype="float32", mean=C.MEAN, stddev=C.STDDEV)
U8_HWC = dict(channels=3, channel_major=False, dtype="uint8")
F32_HWC = dict(channels=3, channel_major=False, bgr_to_rgb=True, dtype="float32", mean=C.MEAN, stddev=C.STDDEV)

CASES = [
    # (name, src (w, h), params kwargs, out kwargs)
    ("up", (256, 256), dict(crop_x=5, crop_y=9, crop_w=200, crop_h=180, out_w=224, out_h=224), F32),
    ("down", (256, 256), dict(crop_x=3, crop_y=1, crop_w=250, crop_h=241, out_w=97, out_h=61), U8_HWC),
    ("mixed_axes", (320, 120), dict(crop_x=10, crop_y=10, crop_w=300, crop_h=100, out_w=150, out_h=200), U8_HWC),
    ("int3x", (400, 300), dict(crop_x=8, crop_y=6, crop_w=384, crop_h=288, out_w=128, out_h=96), U8_HWC),
    ("int2x", (448, 448), dict(crop_x=0, crop_y=0, crop_w=448, crop_h=448, out_w=224, out_h=224, flip=1), F32),
    ("int2x1", (448, 300), dict(crop_x=0, crop_y=0, crop_w=448, crop_h=224, out_w=224, out_h=224), U8_HWC),
    ("int4x3", (400, 300), dict(crop_x=0, crop_y=0, crop_w=400, crop_h=300, out_w=100, out_h=100), U8_HWC),
    ("odd_tail", (333, 217), dict(crop_x=3, crop_y=2, crop_w=301, crop_h=199, out_w=223, out_h=97, flip=1), F32),
    ("tiny_up", (7, 5), dict(crop_x=0, crop_y=0, crop_w=7, crop_h=5, out_w=64, out_h=48), U8_HWC),
    ("one_pixel", (1, 1), dict(crop_x=0, crop_y=0, crop_w=1, crop_h=1, out_w=16, out_h=8), U8_HWC),
    ("narrow", (64, 512), dict(crop_x=0, crop_y=0, crop_w=5, crop_h=512, out_w=3, out_h=100), U8_HWC),
    ("big_down", (2000, 1500), dict(crop_x=100, crop_y=50, crop_w=1800, crop_h=1400, out_w=224, out_h=224), F32),
    ("huge_down", (4096, 3072), dict(crop_x=0, crop_y=0, crop_w=4096, crop_h=3072, out_w=61, out_h=47), U8_HWC),
    ("wide", (1500, 100), dict(crop_x=7, crop_y=3, crop_w=1480, crop_h=90, out_w=1200, out_h=40, flip=1), U8_HWC),
    ("padding_resize", (30, 30), dict(crop_x=0, crop_y=0, crop_w=30, crop_h=30, out_w=64, out_h=48, padding=10,
                                      pad_off_x=20, pad_off_y=0), U8_HWC),
    ("padding_down", (40, 40), dict(crop_x=0, crop_y=0, crop_w=40, crop_h=40, out_w=24, out_h=17, padding=6,
                                    pad_off_x=1, pad_off_y=11), U8_HWC),
    ("photometric", (256, 256), dict(crop_x=3, crop_y=1, crop_w=250, crop_h=241, out_w=224, out_h=224, flip=1,
                                     brightness=0.75, saturation=1.8, contrast=0.65, hue=29,
                                     lighting=[1.5, -2.0, 0.7], color_noise_std=0.1), F32),
    ("resize_short_up", (120, 90), dict(crop_x=40, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                        resize_short_size=256), F32),
    ("resize_short_down", (480, 360), dict(crop_x=50, crop_y=10, crop_w=224, crop_h=224, out_w=224, out_h=224,
                                           resize_short_size=256), F32),
    ("resize_short_then_resize", (500, 375), dict(crop_x=20, crop_y=4, crop_w=300, crop_h=250, out_w=160,
                                                  out_h=128, resize_short_size=300, flip=1), U8_HWC),
    ("rotated", (300, 240), dict(crop_x=20, crop_y=10, crop_w=250, crop_h=200, out_w=160, out_h=120, angle=30), F32),
    # f32 outputs of 341+ columns near 1:1: a 3-channel final_out band needs 3 * ceil(cw / 4) lanes, so
    # its column band must stop at 340 (round-5 advisor: columns 336-340 of channel 2 went unwritten)
    ("wide_f32_384", (400, 300), dict(crop_x=5, crop_y=3, crop_w=390, crop_h=160, out_w=384, out_h=40, flip=1), F32),
    ("wide_f32_512", (520, 200), dict(crop_x=2, crop_y=1, crop_w=515, crop_h=64, out_w=512, out_h=64), F32),
    # resizeArea_ as resize_sep's INTER_AREA form (round 6): K = floor(max scale) + 2 taps -- just under 3
    # (K = 4), just under 7 (K = 8, zero-padded taps reading past the row), just above 7 (resize_generic)
    ("area_k4_edge", (320, 320), dict(crop_x=7, crop_y=3, crop_w=299, crop_h=298, out_w=100, out_h=100, flip=1), F32),
    ("area_k8_edge", (720, 520), dict(crop_x=5, crop_y=9, crop_w=690, crop_h=483, out_w=100, out_h=70), U8_HWC),
    ("area_k8_f32", (720, 520), dict(crop_x=0, crop_y=0, crop_w=689, crop_h=481, out_w=100, out_h=70, flip=1), F32),
    ("area_over_k8", (760, 560), dict(crop_x=3, crop_y=2, crop_w=710, crop_h=500, out_w=100, out_h=70), U8_HWC),
    # identity resizes with f32 output and no photometric stage: through the call's resize class with
    # identity taps (round 6), planes and pixels, flipped, and over add_padding's zero border
    ("identity_f32", (256, 256), dict(crop_x=16, crop_y=9, crop_w=224, crop_h=224, out_w=224, out_h=224, flip=1), F32),
    ("identity_hwc", (300, 200), dict(crop_x=3, crop_y=5, crop_w=221, crop_h=150, out_w=221, out_h=150), F32_HWC),
    ("identity_padded", (40, 30), dict(crop_x=0, crop_y=0, crop_w=40, crop_h=30, out_w=40, out_h=30, padding=6,
                                       pad_off_x=2, pad_off_y=9, flip=1), F32),
]


@pytest.mark.parametrize("method", list(METHODS))
@pytest.mark.parametrize("name,src,pk,ok", CASES, ids=[c[0] for c in CASES])
def test_resize_method_cases(ctx, method, name, src, pk, ok):
    w, h = src
    imgs = [A.synthetic_image(i, w, h, 3) for i in range(3)]
    params = [A.aug_params(interp=METHODS[method], **pk) for _ in imgs]
    stride = pk["out_w"] * pk["out_h"] * 3 * (4 if ok["dtype"] == "float32" else 1)
    out = A.out_desc(item_stride=stride, **ok)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), f"{method} {name}")


@pytest.mark.parametrize("method", list(METHODS))
def test_resize_methods_grayscale(ctx, method):
    imgs = [A.synthetic_image(i, 97, 61, 1) for i in range(4)]
    sizes = [(64, 48), (40, 20), (97, 30), (33, 61)]
    params = [A.aug_params(crop_x=4, crop_y=2, crop_w=80, crop_h=50, out_w=ow, out_h=oh, flip=i % 2,
                           interp=METHODS[method]) for i, (ow, oh) in enumerate(sizes)]
    out = A.out_desc(channels=1, channel_major=True, dtype="uint8", item_stride=97 * 61)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), f"{method} gray")


@pytest.mark.parametrize("method", list(METHODS))
def test_resize_methods_raw_match_cv_resize(ctx, method):
    """Whole-image crop, no augmentation, uint8 HWC out: the output IS cv::resize of the source."""
    import oracle as O
    src = A.synthetic_image(5, 211, 157, 3)
    for ow, oh in ((224, 224), (100, 61), (70, 157), (211, 40), (422, 314)):
        p = A.aug_params(crop_x=0, crop_y=0, crop_w=211, crop_h=157, out_w=ow, out_h=oh, interp=METHODS[method])
        out = A.out_desc(item_stride=ow * oh * 3, **U8_HWC)
        (got,) = H.hip_records(ctx, [src], [p], out)
        assert np.array_equal(got, O.resize(src, ow, oh, method)), (method, ow, oh)


@pytest.mark.parametrize("method", list(METHODS))
def test_resize_methods_c3_pipeline(ctx, method):
    """The C3 augmentation (scale / aspect crops, flips, every photometric stage) with the method set
    in the config, ragged sources, drawn by make_params."""
    aug = dict(C.C3_AUG, interpolation_method=method)
    rng = np.random.default_rng(17)
    imgs = [A.synthetic_image(i, int(rng.integers(200, 520)), int(rng.integers(200, 520)), 3) for i in range(16)]
    params = H.draw_params(aug, [(im.shape[1], im.shape[0]) for im in imgs], 224, 224, seed=23)
    assert all(p.interp == METHODS[method] for p in params)
    out = A.out_desc(item_stride=3 * 224 * 224 * 4, **F32)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), f"{method} C3")


def test_resize_methods_mixed_batch(ctx):
    """One call mixing every method (LINEAR / NEAREST tile groups and the generic pre-pass) and
    resize_short records: each record lands in its own slot."""
    imgs, params = [], []
    codes = [A.INTERP_LINEAR, A.INTERP_NEAREST, A.INTERP_CUBIC, A.INTERP_AREA, A.INTERP_LANCZOS4]
    for i in range(20):
        imgs.append(A.synthetic_image(i, 300 + 7 * i, 260 - 3 * i, 3))
        params.append(A.aug_params(crop_x=i, crop_y=2 * i, crop_w=200 + i, crop_h=180 - i, out_w=224, out_h=224,
                                   flip=i & 1, interp=codes[i % 5], resize_short_size=256 if i % 3 == 0 else 0,
                                   brightness=0.9 if i % 4 == 0 else 1.0))
    out = A.out_desc(item_stride=3 * 224 * 224 * 4, **F32)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "mixed")


@pytest.mark.parametrize("method", list(METHODS))
@pytest.mark.parametrize("case", ["hwc", "gray", "padded", "odd_stride", "no_mean"])
def test_resize_methods_final_output(ctx, method, case):
    """Records with no photometric stage and f32 output: the resize pass writes the loader's layout
    itself (ResizeJob.final_out -- flip, BGR->RGB, the standardize LUT, planes or pixels).  Covers the
    HWC layout, one channel, add_padding's border, item strides that leave the planes' rows off 16-byte
    alignment (element stores instead of float4), and no mean/stddev (the LUT is (float)x)."""
    cn = 1 if case == "gray" else 3
    imgs = [A.synthetic_image(40 + i, 211, 157, cn) for i in range(4)]
    sizes = [(224, 224), (97, 61), (101, 45), (35, 160)]
    pad = dict(padding=8, pad_off_x=3, pad_off_y=12) if case == "padded" else {}
    params = [A.aug_params(crop_x=5 + i, crop_y=3, crop_w=180 - 7 * i, crop_h=140 - 5 * i, out_w=ow, out_h=oh,
                           flip=i % 2, interp=METHODS[method], **pad) for i, (ow, oh) in enumerate(sizes)]
    ok = dict(F32_HWC if case == "hwc" else F32)
    if cn == 1:
        ok.update(channels=1, bgr_to_rgb=False, mean=[0.5], stddev=[0.25])
    if case == "no_mean":
        ok.pop("mean"), ok.pop("stddev")
    stride = 224 * 224 * cn * 4 + (36 if case == "odd_stride" else 0)
    out = A.out_desc(item_stride=stride, **ok)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), f"{method} {case}")


@pytest.mark.parametrize("method", list(METHODS))
def test_resize_c2_batch(ctx, method):
    """A C2 batch of 64 random crops with the method set.  LANCZOS4: its taps are finished on the GPU
    from the host's libm sin / cos (stage.cpp lanczos4_inputs -> resize_kernels.hip lanczos4_taps), as
    many distinct fractions per axis as output columns and rows, against the oracle's taps computed on
    the host from end to end.  AREA: the batch holds both method classes (resizeArea_ records on
    resize_generic, upscaled axes on resize_sep<2>), launched concurrently on the slot's side stream and
    the call's stream."""
    aug = dict(C.C2_AUG, interpolation_method=method)
    imgs = [A.synthetic_image(60 + i, 256, 256, 3) for i in range(64)]
    params = H.draw_params(aug, [(256, 256)] * 64, 224, 224, seed=29)
    assert all(p.interp == METHODS[method] for p in params)
    if method == "AREA":
        down = [p.crop_w >= 224 and p.crop_h >= 224 for p in params]
        assert any(down) and not all(down), "the batch should mix resizeArea_ and bilinear-emulation records"
    out = A.out_desc(item_stride=3 * 224 * 224 * 4, **F32)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), f"{method} C2")


@pytest.mark.parametrize("method", list(METHODS))
def test_resize_shared_axes(ctx, method):
    """Records sharing crop sizes (LANCZOS4: one tap array per distinct axis, stage.cpp GrPlan::axis_taps)
    at different crop positions, flips and source images, mixed with a record of another size and an
    identity record, equal the oracle record by record."""
    imgs = [A.synthetic_image(80 + i, 300, 260, 3) for i in range(9)]
    geo = [(0, 0, 250, 200), (30, 40, 250, 200), (49, 59, 250, 200), (7, 3, 250, 180), (10, 12, 224, 224),
           (3, 3, 250, 200), (50, 60, 250, 200), (11, 5, 190, 230), (2, 9, 250, 200)]
    params = [A.aug_params(crop_x=x, crop_y=y, crop_w=w, crop_h=h, out_w=224, out_h=224, flip=i % 2,
                           interp=METHODS[method]) for i, (x, y, w, h) in enumerate(geo)]
    out = A.out_desc(item_stride=3 * 224 * 224 * 4, **F32)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), f"{method} shared axes")
