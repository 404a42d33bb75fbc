"""GPU parity: the HIP stage (through the C ABI) against aeon's goldens and the CPU oracle.

Bar (BASELINE.json north_star): the uint8 image before standardize is
bit-exact; the fp32 output is compared bit-exactly too (the standardize LUT reproduces
aeon's f64-per-op arithmetic, pinned by the goldens), i.e. tolerance 0 <= 1e-5.
"""
import numpy as np
import pytest

import aeon_amd as A
import oracle as O
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu


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


def _synthetic(n, w=256, h=256, seed=0x5EED, ragged=False):
    rng = np.random.default_rng(7)
    imgs = []
    for i in range(n):
        if ragged:
            w, h = int(rng.integers(256, 513)), int(rng.integers(256, 513))
        imgs.append(A.synthetic_image(i, w, h, 3, seed))
    return imgs


MEAN_OUT = dict(channels=3, channel_major=True, bgr_to_rgb=True, dtype="float32",
                mean=C.MEAN, stddev=C.STDDEV, item_stride=3 * 224 * 224 * 4)


def test_golden_train(ctx, golden):
    """provider.image_paddle_imagenet_training_augmentation (test/test_provider.cpp:96-177)."""
    p = A.aug_params(crop_x=50, crop_y=50, crop_w=171, crop_h=201, out_w=224, out_h=224, flip=1)
    out = A.out_desc(**MEAN_OUT)
    (res,) = H.hip_records(ctx, [golden["img"]], [p], out)
    assert np.array_equal(res, golden["train"])


def test_golden_eval(ctx, golden):
    """provider.image_paddle_imagenet_validate_augmentation (test/test_provider.cpp:179-261):
    resize_short 256 -> center crop 224 (the C1 configuration)."""
    (p,) = H.draw_params(C.C1_AUG, [(480, 360)], 224, 224)
    out = A.out_desc(**MEAN_OUT)
    (res,) = H.hip_records(ctx, [golden["img"]], [p], out)
    assert np.array_equal(res, golden["eval"])


@pytest.mark.parametrize("aug_name", ["C1", "C2", "C3"])
def test_configs_fixed_256(ctx, aug_name):
    aug = {"C1": C.C1_AUG, "C2": C.C2_AUG, "C3": C.C3_AUG}[aug_name]
    imgs = _synthetic(24)
    params = H.draw_params(aug, [(256, 256)] * len(imgs), 224, 224, seed=3)
    out = A.out_desc(**MEAN_OUT)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), aug_name)


def test_c3_ragged(ctx):
    imgs = _synthetic(24, ragged=True)
    params = H.draw_params(C.C3_AUG, [(im.shape[1], im.shape[0]) for im in imgs], 224, 224, seed=11)
    out = A.out_desc(**MEAN_OUT)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "C3 ragged")


def test_real_image_c3(ctx, golden):
    imgs = [golden["img"]] * 16
    params = H.draw_params(C.C3_AUG, [(480, 360)] * 16, 224, 224, seed=5)
    out = A.out_desc(**MEAN_OUT)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "C3 real")


def test_c5_image_and_mask(ctx):
    """etl [image 512, pixelmask 512]: the mask shares the image's params (provider.cpp:378-391)."""
    rng = np.random.default_rng(3)
    imgs, masks = [], []
    for i in range(8):
        w, h = int(rng.integers(300, 700)), int(rng.integers(300, 700))
        imgs.append(A.synthetic_image(i, w, h, 3))
        masks.append(((A.synthetic_image(100 + i, w, h, 1) > 127) * 255).astype(np.uint8))
    params = H.draw_params(C.C5_AUG, [(im.shape[1], im.shape[0]) for im in imgs], 512, 512, seed=9)
    iout = C.out_desc_for(C.IMAGE_512, C.C5_AUG)
    mout = C.out_desc_for(C.MASK_512, C.C5_AUG)
    _assert_same(H.hip_records(ctx, imgs, params, iout), H.oracle_records(imgs, params, iout), "C5 image")
    mres = H.hip_records(ctx, masks, params, mout, mask=True)
    _assert_same(mres, H.oracle_records(masks, params, mout, mask=True), "C5 mask")
    for m in mres:  # test/test_pixel_mask.cpp invariant: NEAREST keeps only the source values
        assert set(np.unique(m)) <= {0, 255}


@pytest.mark.parametrize("channel_major", [True, False])
def test_fixed_aspect_ratio_canvas(ctx, channel_major):
    """image::loader with fixed_aspect_ratio (etl_image.cpp:258-306) after crop_enable=false
    params (augment_image.cpp:132-151: the record scaled to fit, image.var_resize_fixed_ratio
    300x200 -> 400x267, test/test_image.cpp:1070-1100): the record at the top-left of a zeroed
    canvas; the pixelmask shares the params and the loader (provider.cpp:353-391)."""
    aug = {"type": "image", "fixed_aspect_ratio": True, "crop_enable": False, "flip_enable": True}
    etl = {"type": "image", "height": 400, "width": 400, "channels": 3, "output_type": "uint8_t",
           "channel_major": channel_major, "bgr_to_rgb": True}
    metl = {"type": "pixelmask", "height": 400, "width": 400, "channels": 1, "output_type": "uint8_t",
            "channel_major": channel_major}
    sizes = [(300, 200), (200, 300), (400, 400), (123, 457), (640, 480), (31, 17), (801, 399)]
    imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
    masks = [A.synthetic_image(50 + i, w, h, 1) for i, (w, h) in enumerate(sizes)]
    params = H.draw_params(aug, sizes, 400, 400, seed=4)
    assert (params[0].out_w, params[0].out_h) == (400, 267)
    assert any(p.flip for p in params) and any(not p.flip for p in params)
    out, mout = C.out_desc_for(etl, aug), C.out_desc_for(metl, aug)
    ref = [H.place_canvas(r, out) for r in H.oracle_records(imgs, params, out)]
    _assert_same(H.hip_canvases(ctx, imgs, params, out), ref, "fixed_aspect image")
    mref = [H.place_canvas(r, mout) for r in H.oracle_records(masks, params, mout, mask=True)]
    _assert_same(H.hip_canvases(ctx, masks, params, mout, mask=True), mref, "fixed_aspect mask")


@pytest.mark.parametrize("otype", ["float", "double", "int32_t"])
@pytest.mark.parametrize("with_mean", [False, True])
@pytest.mark.parametrize("channel_major", [True, False])
def test_fixed_aspect_ratio_non_uint8(ctx, otype, with_mean, channel_major):
    """fixed_aspect_ratio with a non-uint8 output_type (etl_image.cpp:258-306): aeon zeroes the
    item's whole byte size, writes the record as CV_8U planes / pixels at the top-left of the
    canvas whatever the declared type, and standardizes that uint8 canvas in place (OpenCV 2.4
    8-bit arithm_op rules, oracle orc_u8_standardize_value -- parity unpinned)."""
    import oracle as O
    if with_mean and otype == "int32_t":
        pytest.skip("mean/stddev need float or double output")
    aug = {"type": "image", "fixed_aspect_ratio": True, "crop_enable": False, "flip_enable": True}
    if with_mean:
        aug.update(mean=[0.485, 0.456, 0.6], stddev=[0.229, 0.0, 0.225])
    etl = {"type": "image", "height": 96, "width": 128, "channels": 3, "output_type": otype,
           "channel_major": channel_major, "bgr_to_rgb": True}
    sizes = [(64, 40), (200, 90), (128, 96), (31, 77)]
    imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
    params = H.draw_params(aug, sizes, 128, 96, seed=6)
    out = C.out_desc_for(etl, aug)
    u8 = A.out_desc(channels=3, channel_major=channel_major, bgr_to_rgb=True, dtype="uint8",
                    item_stride=128 * 96 * 3, fixed_aspect_ratio=True, canvas=(128, 96))
    canv = [H.place_canvas(r, u8) for r in H.oracle_records(imgs, params, u8)]
    if with_mean:
        lut = np.array([[O.u8_standardize(x, aug["mean"][c], aug["stddev"][c]) for x in range(256)]
                        for c in range(3)], np.uint8)
        for k, cv in enumerate(canv):  # the record's pixels only: the rest of the canvas is 0 -> f(0)
            cm = cv if channel_major else cv.transpose(2, 0, 1)
            for c in range(3):
                cm[c] = lut[c][cm[c]]
            canv[k] = cm if channel_major else cm.transpose(1, 2, 0)
    import torch
    arena, descs = A.pack_images(imgs)
    src = torch.from_numpy(arena).to("cuda")
    dst = torch.full((len(imgs) * out.item_stride,), 0xAB, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ctx.augment_batch(descs, src.data_ptr(), params, out, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    host = dst.cpu().numpy()
    for i, cv in enumerate(canv):
        item = host[i * out.item_stride:(i + 1) * out.item_stride]
        want = np.zeros(out.item_stride, np.uint8)
        want[:cv.size] = np.ascontiguousarray(cv).reshape(-1)
        assert np.array_equal(item, want), (otype, with_mean, channel_major, i)


OUTPUT_TYPES = ["int8_t", "char", "int16_t", "uint16_t", "int32_t", "uint32_t", "double", "float", "uint8_t"]


@pytest.mark.parametrize("otype", OUTPUT_TYPES)
@pytest.mark.parametrize("channel_major", [True, False])
def test_output_types_images(ctx, otype, channel_major):
    """image::loader to every aeon output_type (convert_mix_channels: saturating convertTo of the
    uint8 record, image.cpp:176-212; typemap.hpp:43-52), against the oracle."""
    etl = {"type": "image", "height": 96, "width": 80, "channels": 3, "output_type": otype,
           "channel_major": channel_major, "bgr_to_rgb": True}
    aug = dict(C.C3_AUG)
    if otype not in ("float", "double"):
        aug.pop("mean"), aug.pop("stddev")
    sizes = [(160, 120), (97, 203), (300, 300)]
    imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
    params = H.draw_params(aug, sizes, 80, 96, seed=2)
    out = C.out_desc_for(etl, aug)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), otype)


@pytest.mark.parametrize("otype", OUTPUT_TYPES)
def test_output_types_masks(ctx, otype):
    """pixelmask loader to every output_type (aeon's own int32 masks among them) through the
    NEAREST gather pass and, rotated, through the tile kernel."""
    etl = {"type": "pixelmask", "height": 64, "width": 72, "channels": 1, "output_type": otype}
    sizes = [(100, 90), (64, 72), (333, 111)]
    masks = [(A.synthetic_image(40 + i, w, h, 1) % 37).astype(np.uint8) for i, (w, h) in enumerate(sizes)]
    params = H.draw_params(dict(C.C5_AUG, angle=[-30, 30]), sizes, 72, 64, seed=13)
    out = C.out_desc_for(etl, C.C5_AUG)
    _assert_same(H.hip_records(ctx, masks, params, out, mask=True),
                 H.oracle_records(masks, params, out, mask=True), otype)
    for p in params:
        p.angle = 0
    _assert_same(H.hip_records(ctx, masks, params, out, mask=True),
                 H.oracle_records(masks, params, out, mask=True), otype + " unrotated")


# ---- image::rotate (angle != 0) --------------------------------------------------------------
@pytest.mark.parametrize("aug_name", ["C1", "C2", "C3"])
def test_rotation_configs(ctx, aug_name):
    # "angle": [-20, 20] as aeon's own image test config (test/test_image.cpp:197)
    aug = dict({"C1": C.C1_AUG, "C2": C.C2_AUG, "C3": C.C3_AUG}[aug_name], angle=[-20, 20])
    imgs = _synthetic(16, ragged=True)
    params = H.draw_params(aug, [(im.shape[1], im.shape[0]) for im in imgs], 224, 224, seed=21)
    assert any(p.angle != 0 for p in params)
    out = A.out_desc(**MEAN_OUT)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), aug_name + " rot")


@pytest.mark.parametrize("angle", [45, -90, 180, 7, 359])
def test_rotation_image_and_mask_fixed_angles(ctx, angle):
    rng = np.random.default_rng(angle & 0xff)
    w, h = int(rng.integers(200, 400)), int(rng.integers(200, 400))
    img = A.synthetic_image(abs(angle) + 7, w, h, 3)
    msk = np.zeros((h, w), np.uint8)
    msk[h // 4:h // 2, w // 5:w // 2] = 3
    msk[h // 2:, w // 3:] = 9
    p = A.aug_params(crop_x=w // 8, crop_y=h // 8, crop_w=w - w // 4, crop_h=h - h // 4, out_w=224, out_h=224,
                     angle=angle, flip=1)
    iout = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
    mout = A.out_desc(channels=1, dtype="uint8", item_stride=224 * 224)
    _assert_same(H.hip_records(ctx, [img], [p], iout), H.oracle_records([img], [p], iout), f"rot {angle}")
    (m,) = H.hip_records(ctx, [msk], [p], mout, mask=True)
    _assert_same([m], H.oracle_records([msk], [p], mout, mask=True), f"mask rot {angle}")
    assert set(np.unique(m)) <= {0, 3, 9}  # test/test_pixel_mask.cpp:130-155 invariant


EDGE_CASES = [
    # (name, src (w,h), params kwargs, out kwargs)
    ("upscale_tiny", (7, 5), dict(crop_x=0, crop_y=0, crop_w=7, crop_h=5, out_w=224, out_h=224), {}),
    ("one_pixel", (1, 1), dict(crop_x=0, crop_y=0, crop_w=1, crop_h=1, out_w=16, out_h=8), {}),
    ("area2x", (448, 448), dict(crop_x=0, crop_y=0, crop_w=448, crop_h=448, out_w=224, out_h=224), {}),
    ("area2x_flip", (500, 480), dict(crop_x=10, crop_y=7, crop_w=448, crop_h=448, out_w=224, out_h=224, flip=1), {}),
    ("copy", (300, 300), dict(crop_x=13, crop_y=21, crop_w=224, crop_h=224, out_w=224, out_h=224), {}),
    ("odd_width_tail", (333, 217), dict(crop_x=3, crop_y=2, crop_w=301, crop_h=199, out_w=223, out_h=97), {}),
    ("narrow", (64, 512), dict(crop_x=0, crop_y=0, crop_w=5, crop_h=512, out_w=3, out_h=100), {}),
    ("huge_downscale", (2000, 1500), dict(crop_x=100, crop_y=50, crop_w=1800, crop_h=1400, out_w=224, out_h=224), {}),
    ("u8_hwc", (256, 256), dict(crop_x=5, crop_y=9, crop_w=200, crop_h=180, out_w=224, out_h=224, flip=1),
     dict(dtype="uint8", channel_major=False, mean=None, stddev=None, item_stride=224 * 224 * 3)),
    ("u8_chw_bgr", (256, 256), dict(crop_x=5, crop_y=9, crop_w=200, crop_h=180, out_w=224, out_h=224),
     dict(dtype="uint8", bgr_to_rgb=False, mean=None, stddev=None, item_stride=224 * 224 * 3)),
    ("f32_hwc_mean", (256, 256), dict(crop_x=5, crop_y=9, crop_w=200, crop_h=180, out_w=224, out_h=224),
     dict(channel_major=False)),
    ("f32_nomean", (256, 256), dict(crop_x=5, crop_y=9, crop_w=200, crop_h=180, out_w=224, out_h=224),
     dict(mean=None, stddev=None)),
    ("brightness_diag", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                         brightness=0.6), {}),
    # x*0.5 and x*1.5 land exactly on .5 for odd x: saturate_cast's round-half-to-even (aeon's
    # brightness KAT: 127*1.5 -> 190)
    ("brightness_ties_half", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                              brightness=0.5), {}),
    ("brightness_ties_1_5", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                             brightness=1.5), {}),
    ("saturation0", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                     saturation=0.0, brightness=0.9), {}),
    ("saturation_float_path", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224,
                                               out_h=224, saturation=40.0), {}),
    ("hue_neg", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224, hue=-179), {}),
    ("hue_pos", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224, hue=180), {}),
    # hue wraps: |hue| < 180 (one conditional subtraction, negative H stored as uchar) and the rest
    ("hue_179", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224, hue=179), {}),
    ("hue_m1_sat", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224, hue=-1,
                                    saturation=1.7), {}),
    ("hue_m180_contrast", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                           hue=-180, contrast=0.8), {}),
    ("hue_401", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224, hue=401), {}),
    ("hue_m397", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224, hue=-397), {}),
    ("contrast_only", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                       contrast=0.3), {}),
    ("lighting_only", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                       lighting=[1.5, -2.0, 0.7], color_noise_std=0.1), {}),
    ("nearest_interp", (256, 256), dict(crop_x=3, crop_y=3, crop_w=190, crop_h=211, out_w=224, out_h=224,
                                        interp=1), {}),
    ("padding", (32, 32), dict(crop_x=0, crop_y=0, crop_w=32, crop_h=32, out_w=32, out_h=32, padding=5,
                               pad_off_x=2, pad_off_y=8), dict(item_stride=3 * 32 * 32 * 4)),
    ("padding_resize", (30, 30), dict(crop_x=0, crop_y=0, crop_w=30, crop_h=30, out_w=64, out_h=48, padding=10,
                                      pad_off_x=20, pad_off_y=0), dict(item_stride=3 * 64 * 48 * 4)),
    ("resize_short_upscale", (120, 90), dict(crop_x=40, crop_y=0, crop_w=256, crop_h=256, out_w=224, out_h=224,
                                             resize_short_size=256), {}),
    # maximum sizes: outputs wider than a workgroup's column groups, 12-megapixel sources
    ("wide_output", (1500, 100), dict(crop_x=7, crop_y=3, crop_w=1480, crop_h=90, out_w=1200, out_h=40, flip=1),
     dict(item_stride=3 * 1200 * 40 * 4)),
    ("very_wide_output", (1300, 40), dict(crop_x=0, crop_y=0, crop_w=1300, crop_h=40, out_w=2500, out_h=16),
     dict(item_stride=3 * 2500 * 16 * 4)),
    ("big_source", (4096, 3072), dict(crop_x=11, crop_y=5, crop_w=4000, crop_h=3000, out_w=512, out_h=384, flip=1),
     dict(item_stride=3 * 512 * 384 * 4)),
    ("big_source_c3", (4096, 3072), dict(crop_x=0, crop_y=0, crop_w=4096, crop_h=3072, out_w=224, out_h=224,
                                         brightness=0.7, saturation=1.6, contrast=0.6, hue=9), {}),
    # a contrast record of more than 2^32 / 255 pixels: its channel sums need 64 bits (contrast_reduce)
    ("contrast_u64_sums", (1030, 16400), dict(crop_x=0, crop_y=0, crop_w=1030, crop_h=16400, out_w=1030,
                                              out_h=16400, contrast=0.6, brightness=1.2),
     dict(item_stride=3 * 1030 * 16400 * 4)),
    # uint8 planes: 4-byte groups stored as dwords when aligned, bytewise when the plane's rows are not
    ("u8_chw_odd_width", (256, 256), dict(crop_x=5, crop_y=9, crop_w=200, crop_h=180, out_w=221, out_h=37, flip=1),
     dict(dtype="uint8", mean=None, stddev=None, item_stride=221 * 37 * 3)),
    ("u8_chw_c3_odd", (256, 256), dict(crop_x=0, crop_y=0, crop_w=256, crop_h=256, out_w=223, out_h=31,
                                      brightness=0.8, saturation=1.3, contrast=0.7, hue=-12),
     dict(dtype="uint8", mean=None, stddev=None, item_stride=223 * 31 * 3)),
] + [
    # contrast pass 1's specialised loop (fixed-point brightness/saturation + hue, packed HSV2RGB
    # with the per-H channel selector): every hue wrap, sector boundaries included
    (f"spec_bs_hue_{hue}", (256, 256), dict(crop_x=3, crop_y=1, crop_w=250, crop_h=241, out_w=224, out_h=224,
                                            flip=hue & 1, brightness=0.75, saturation=1.8, contrast=0.65, hue=hue),
     {}) for hue in (-397, -180, -179, -91, -30, -1, 1, 29, 30, 90, 150, 179, 180, 401)
]


@pytest.mark.parametrize("name,src,pk,ok", EDGE_CASES, ids=[c[0] for c in EDGE_CASES])
def test_edge_cases(ctx, name, src, pk, ok):
    w, h = src
    imgs = [A.synthetic_image(i, w, h, 3) for i in range(3)]
    params = [A.aug_params(**pk) for _ in imgs]
    kw = dict(MEAN_OUT)
    kw.update(ok)
    out = A.out_desc(**kw)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), name)


def test_grayscale(ctx):
    imgs = [A.synthetic_image(i, 97, 61, 1) for i in range(4)]
    params = [A.aug_params(crop_x=4, crop_y=2, crop_w=80, crop_h=50, out_w=64, out_h=48, flip=i % 2)
              for i in range(4)]
    out = A.out_desc(channels=1, channel_major=True, dtype="uint8", item_stride=64 * 48)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "gray")


@pytest.mark.parametrize("ow,oh", [(64, 48), (61, 47), (510, 3)])
def test_mask_u8_widths(ctx, ow, oh):
    """1-channel uint8 output rows of any width (dword stores only on aligned 4-byte groups)."""
    masks = [A.synthetic_image(30 + i, 97, 61, 1) for i in range(4)]
    params = [A.aug_params(crop_x=3, crop_y=1, crop_w=90, crop_h=57, out_w=ow, out_h=oh, flip=i % 2)
              for i in range(4)]
    out = A.out_desc(channels=1, channel_major=True, dtype="uint8", item_stride=ow * oh)
    res = H.hip_records(ctx, masks, params, out, mask=True)
    _assert_same(res, H.oracle_records(masks, params, out, mask=True), f"mask {ow}x{oh}")


def test_empty_batch(ctx):
    import torch
    out = A.out_desc(**MEAN_OUT)
    buf = torch.zeros(16, dtype=torch.uint8, device="cuda")
    ctx.augment_batch([], buf.data_ptr(), [], out, buf.data_ptr())
    ctx.synchronize()


def test_errors(ctx):
    img = A.synthetic_image(0, 64, 64)
    out = A.out_desc(**MEAN_OUT)
    with pytest.raises(A.AeonHipError) as e:  # no cv::INTER_* value 9
        H.hip_records(ctx, [img], [A.aug_params(crop_w=64, crop_h=64, out_w=224, out_h=224, interp=9)], out)
    assert e.value.code == A.AEON_HIP_EINVAL
    bad = A.out_desc(**MEAN_OUT)
    bad.dtype = 99
    with pytest.raises(A.AeonHipError) as e:
        H.hip_records(ctx, [img], [A.aug_params(crop_w=64, crop_h=64, out_w=224, out_h=224)], bad)
    assert e.value.code == A.AEON_HIP_EUNSUPPORTED
    with pytest.raises(A.AeonHipError) as e:
        H.hip_records(ctx, [img], [A.aug_params(crop_x=10, crop_w=64, crop_h=64, out_w=224, out_h=224)], out)
    assert e.value.code == A.AEON_HIP_EINVAL


def _oracle_batch(imgs, params, out, shape):
    """The oracle's threaded batch entry (orc_batch_augment, aeon's pool policy) over every record."""
    import os
    lc = H.oracle_load_config(out)
    res, _ = O.batch_augment(imgs, [H.to_oracle_params(p) for p in params], lc, shape,
                             min(16, os.cpu_count() or 1))
    return list(res)


def test_full_batch_c3_all_records(ctx):
    """BASELINE.json C3 at its full size (batch 1024, 224x224 fp32): contrast pass 1 + reduce +
    pass 2, both on persistent grids whose last rounds come from the dynamic-tail counter (most of
    pass 1's tiles past the first round are drawn).  Every record against the oracle; a rerun is
    bit-identical (the counter hands the tail tiles to other workgroups each time)."""
    n = 1024
    imgs = _synthetic(n)
    params = H.draw_params(C.C3_AUG, [(256, 256)] * n, 224, 224, seed=1)
    out = A.out_desc(**MEAN_OUT)
    r1 = H.hip_records(ctx, imgs, params, out)
    r2 = H.hip_records(ctx, imgs, params, out)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r2)), "C3 rerun differs"
    _assert_same(r1, _oracle_batch(imgs, params, out, (3, 224, 224)), "C3 full batch")


@pytest.mark.parametrize("node_id", [1, 7])
def test_c4_rank_window(node_id):
    """C4 = C3 sharded over 8 GPUs: rank g decodes its manifest slice (manifest_file.cpp:278-295)
    with the decoder seeded random_seed + node_id (loader.cpp:174, batch_decoder.cpp:47-54).  One
    per-GPU batch of 1024 records of rank `node_id` of 8 through aeon_decoder, every record against
    the oracle with the checker's own slot engines seeded 1 + node_id."""
    n_global, batch, ranks = 8192, 1024, 8
    idx = A.manifest_node_slice(n_global, batch, node_id, ranks)
    assert len(idx) == batch
    recs = [(A.synthetic_image(int(i), 256, 256, 3),) for i in idx]
    cfg = dict(batch_size=batch, random_seed=1, node_id=node_id, node_count=ranks, etl=[C.IMAGE_224],
               augmentation=[C.C3_AUG])
    d = A.Decoder(cfg)
    try:
        (got,) = d.decode(recs)
    finally:
        d.close()
    params = H.draw_params(C.C3_AUG, [(256, 256)] * batch, 224, 224, seed=1 + node_id)
    out = C.out_desc_for(C.IMAGE_224, C.C3_AUG)
    ref = _oracle_batch([r[0] for r in recs], params, out, (3, 224, 224))
    _assert_same(list(got), ref, f"C4 rank {node_id}")


def test_full_batch_c2_all_records(ctx):
    """BASELINE.json C2 at its headline size: 256 records of 256x256 -> 224x224 fp32 CHW is 1,792
    tiles on a persistent grid of 768 workgroups, so every workgroup walks 2-3 tiles (the
    multi-tile staging path every headline number runs).  All 256 records bit-exact against the
    oracle (test/test_provider.cpp:96-177 semantics, per record); a rerun is bit-identical."""
    n = 256
    imgs = _synthetic(n)
    params = H.draw_params(C.C2_AUG, [(256, 256)] * n, 224, 224, seed=1)
    out = A.out_desc(**MEAN_OUT)
    r1 = H.hip_records(ctx, imgs, params, out)
    r2 = H.hip_records(ctx, imgs, params, out)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r2)), "C2 rerun differs"
    _assert_same(r1, H.oracle_records(imgs, params, out), "C2 full batch")


def test_full_batch_c5_all_records(ctx):
    """BASELINE.json C5 at its size: 128 image + pixel-mask pairs, 640x480 sources -> 512x512
    (image bilinear fp32 CHW, mask NEAREST uint8), shared params; every record of both against
    the oracle, plus a bit-identical rerun."""
    n = 128
    rng = np.random.default_rng(55)
    imgs = [A.synthetic_image(i, 640, 480, 3) for i in range(n)]
    masks = [rng.integers(0, 21, (480, 640), dtype=np.uint8) for _ in range(n)]
    params = H.draw_params(C.C5_AUG, [(640, 480)] * n, 512, 512, seed=1)
    iout = C.out_desc_for(C.IMAGE_512, C.C5_AUG)
    mout = C.out_desc_for(C.MASK_512, C.C5_AUG)
    i1 = H.hip_records(ctx, imgs, params, iout)
    m1 = H.hip_records(ctx, masks, params, mout, mask=True)
    i2 = H.hip_records(ctx, imgs, params, iout)
    m2 = H.hip_records(ctx, masks, params, mout, mask=True)
    assert all(np.array_equal(a, b) for a, b in zip(i1 + m1, i2 + m2)), "C5 rerun differs"
    _assert_same(i1, H.oracle_records(imgs, params, iout), "C5 image full batch")
    _assert_same(m1, H.oracle_records(masks, params, mout, mask=True), "C5 mask full batch")


@pytest.mark.parametrize("cfg", ["C2", "C3", "C5_mask", "fixed_u8"])
def test_zero_copy_host_buffers(ctx, cfg):
    """Outputs stored straight into pinned host memory by the kernels (out_dev = a device-mapped
    pinned buffer: the zero-copy host->host path, tools/e2e_probe.py), and sources read from pinned
    host memory, give exactly the device-resident call's bytes -- single-pass, contrast two-pass,
    the mask gather pass, and fixed_aspect_ratio (whose canvas fill is a memset on the host buffer)."""
    import torch
    n = 24
    mask = cfg == "C5_mask"
    if mask:
        rng = np.random.default_rng(3)
        imgs = [rng.integers(0, 21, (480, 640), dtype=np.uint8) for _ in range(n)]
        params = H.draw_params(C.C5_AUG, [(640, 480)] * n, 512, 512, seed=2)
        out = C.out_desc_for(C.MASK_512, C.C5_AUG)
    elif cfg == "fixed_u8":
        aug = {"type": "image", "fixed_aspect_ratio": True, "crop_enable": False, "flip_enable": True}
        etl = {"type": "image", "height": 96, "width": 128, "channels": 3, "output_type": "uint8_t",
               "channel_major": True}
        sizes = [(64 + 7 * i, 40 + 5 * i) for i in range(n)]
        imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
        params = H.draw_params(aug, sizes, 128, 96, seed=6)
        out = C.out_desc_for(etl, aug)
    else:
        aug = C.C2_AUG if cfg == "C2" else C.C3_AUG
        imgs = _synthetic(n)
        params = H.draw_params(aug, [(256, 256)] * n, 224, 224, seed=4)
        out = C.out_desc_for(C.IMAGE_224, aug)
    arena, descs = A.pack_images(imgs)
    run = ctx.mask_batch if mask else ctx.augment_batch
    stream = torch.cuda.current_stream().cuda_stream
    src_dev = torch.from_numpy(arena).to("cuda")
    dst_dev = torch.full((n * out.item_stride,), 0xAB, dtype=torch.uint8, device="cuda")
    run(descs, src_dev.data_ptr(), params, out, dst_dev.data_ptr(), stream)
    src_host = torch.from_numpy(arena).pin_memory()
    for src in (src_dev, src_host):
        dst_host = torch.full((n * out.item_stride,), 0xCD, dtype=torch.uint8).pin_memory()
        run(descs, src.data_ptr(), params, out, dst_host.data_ptr(), stream)
        ctx.synchronize(stream)
        assert torch.equal(dst_host, dst_dev.cpu()), (cfg, "host source" if src is src_host else "device source")


@pytest.mark.parametrize("aug_name", ["C2", "C3_no_contrast", "C5_image", "nearest_u8"])
def test_direct_jobs_match_device_table(ctx, monkeypatch, aug_name):
    """run_direct (the tile kernel reading its jobs from the caller's pinned slot over PCIe) against
    the multi-pass path with the job table uploaded to the device (AEON_HIP_DIRECT=0) and the oracle:
    same outputs, bit for bit, for every single-pass record shape (bilinear, photometric without
    contrast, nearest / uint8 HWC)."""
    aug = {"C2": C.C2_AUG, "C3_no_contrast": dict(C.C3_AUG, contrast=[1.0, 1.0]), "C5_image": C.C5_AUG,
           "nearest_u8": dict(C.C2_AUG, interpolation_method="NEAREST")}[aug_name]
    ow, oh = (512, 512) if aug_name == "C5_image" else (224, 224)
    rng = np.random.default_rng(77)
    sizes = [(int(rng.integers(200, 700)), int(rng.integers(200, 700))) for _ in range(40)]
    imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
    params = H.draw_params(aug, sizes, ow, oh, seed=8)
    if aug_name == "nearest_u8":
        out = A.out_desc(channels=3, channel_major=False, dtype="uint8", item_stride=ow * oh * 3)
    else:
        out = A.out_desc(**dict(MEAN_OUT, item_stride=3 * ow * oh * 4))
    dev = H.hip_records(ctx, imgs, params, out)
    monkeypatch.setenv("AEON_HIP_DIRECT", "0")
    host_ctx = A.Context(0)
    host = H.hip_records(host_ctx, imgs, params, out)
    host_ctx.close()
    _assert_same(dev, host, aug_name + " direct vs device job table")
    _assert_same(dev, H.oracle_records(imgs, params, out), aug_name)


def test_mask_rejects_standardize(ctx):
    """pixel_mask's loader never standardizes (etl_pixel_mask.cpp:94-105): refused either way."""
    m = A.synthetic_image(0, 64, 64, 1)
    p = A.aug_params(crop_x=0, crop_y=0, crop_w=64, crop_h=64, out_w=32, out_h=32)
    out = A.out_desc(channels=1, dtype="float32", mean=(0.5,), stddev=(0.2,), item_stride=32 * 32 * 4)
    for angle in (0, 30):
        p.angle = angle
        with pytest.raises(A.AeonHipError, match="no mean/stddev"):
            H.hip_records(ctx, [m], [p], out, mask=True)


# ---- batch transpose (batch_major=false layout) ---------------------------------------------
@pytest.mark.parametrize("rows,cols,esize", [(256, 150528, 4), (7, 1000, 4), (64, 64, 4), (1, 33, 4),
                                             (33, 1, 4), (5, 127, 1), (130, 70, 2), (3, 65, 8)])
def test_transpose_batch_matches_oracle(rows, cols, esize):
    import torch
    import oracle as O
    n = rows * cols * esize
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    dst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ctx = A.Context(0)
    st = torch.cuda.current_stream().cuda_stream
    ctx.transpose_batch(src.data_ptr(), dst.data_ptr(), rows, cols, esize, st)
    ctx.synchronize(st)
    ref = O.transpose(src.cpu().numpy(), rows, cols, esize)
    assert np.array_equal(dst.cpu().numpy(), ref)
    ctx.close()


def test_transpose_batch_rejects_bad_arguments():
    import torch
    src = torch.zeros(64, dtype=torch.uint8, device="cuda")
    ctx = A.Context(0)
    with pytest.raises(A.AeonHipError, match="unsupported datatype"):
        ctx.transpose_batch(src.data_ptr(), src.data_ptr() + 32, 2, 2, 3)
    with pytest.raises(A.AeonHipError, match="overlap"):
        ctx.transpose_batch(src.data_ptr(), src.data_ptr() + 8, 4, 4, 1)
    ctx.close()


def _pack16(masks):
    """16-bit single-channel records -> (uint8 arena, ImgDesc with elem_bytes=2)."""
    chunks, descs, off = [], [], 0
    for m in masks:
        b = np.ascontiguousarray(m, dtype="<u2").view(np.uint8).reshape(-1)
        pad = (-len(b)) % 16
        chunks.append(np.concatenate([b, np.zeros(pad, np.uint8)]))
        h, w = m.shape
        descs.append(A.ImgDesc(offset=off, width=w, height=h, stride=2 * w, channels=1, elem_bytes=2))
        off += len(b) + pad
    return np.concatenate(chunks), (A.ImgDesc * len(descs))(*descs)


@pytest.mark.parametrize("dtype", ["uint8", "float32", "int8", "int16", "uint16", "int32", "float64"])
@pytest.mark.parametrize("entry", ["mask", "depthmap"])
@pytest.mark.parametrize("rotated", [False, True])
def test_16bit_masks_and_depthmaps(ctx, dtype, entry, rotated):
    """ANYDEPTH records (etl_pixel_mask.cpp:35, etl_depthmap.cpp:35) stay 16-bit through
    crop -> NEAREST -> flip and are converted by the loader (saturate_cast<uchar> / exact float).
    NEAREST is a pure gather, so the oracle reference is its 8-bit transform of the low and high
    byte planes recombined (parity unpinned by aeon's own fixtures: none are 16-bit)."""
    import torch
    rng = np.random.default_rng(16)
    sizes = [(int(rng.integers(40, 300)), int(rng.integers(40, 300))) for _ in range(9)]
    masks = [rng.integers(0, 65536, (h, w), dtype=np.uint16) for w, h in sizes]
    masks[0][:] = rng.integers(0, 256, masks[0].shape)  # values within uint8 too
    params = H.draw_params(dict(C.C5_AUG, angle=[-40, 40]) if rotated else C.C5_AUG, sizes, 128, 96, seed=12)
    assert rotated == any(p.angle != 0 for p in params)
    npt = A.DTYPES[dtype][1]
    esz = np.dtype(npt).itemsize
    out = A.out_desc(channels=1, channel_major=True, dtype=dtype, item_stride=128 * 96 * esz)
    arena, descs = _pack16(masks)
    src = torch.from_numpy(arena).to("cuda")
    dst = torch.full((len(masks) * out.item_stride,), 0x5A, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    getattr(ctx, entry + "_batch")(descs, src.data_ptr(), params, out, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    host = dst.cpu().numpy()
    o8 = A.out_desc(channels=1, channel_major=True, dtype="uint8", item_stride=128 * 96)
    lo = H.oracle_records([(m & 0xff).astype(np.uint8) for m in masks], params, o8, mask=True)
    hi = H.oracle_records([(m >> 8).astype(np.uint8) for m in masks], params, o8, mask=True)
    for i, p in enumerate(params):
        v = hi[i].astype(np.uint32) * 256 + lo[i]
        sat = {"uint8": 255, "int8": 127, "int16": 32767}.get(dtype)  # saturate_cast from CV_16U
        want = (np.minimum(v, sat) if sat else v).astype(npt)
        got = host[i * out.item_stride: i * out.item_stride + v.size * esz].view(want.dtype).reshape(v.shape)
        assert np.array_equal(got, want), (entry, dtype, i)


def test_16bit_errors(ctx):
    import torch
    m = np.zeros((20, 30), np.uint16)
    arena, descs = _pack16([m])
    src = torch.from_numpy(arena).to("cuda")
    dst = torch.zeros(64 * 64, dtype=torch.uint8, device="cuda")
    out = A.out_desc(channels=1, dtype="uint8", item_stride=64 * 64)
    (p,) = H.draw_params(C.C5_AUG, [(30, 20)], 64, 64)
    with pytest.raises(A.AeonHipError, match="pixel masks / depth maps only"):
        ctx.augment_batch(descs, src.data_ptr(), [p], out, dst.data_ptr())



def test_ssd_expand_records(ctx):
    """make_ssd_params records (expand + batch-sampler crop + photometric, "use warping" 300x300):
    image::expand (image.cpp:276-303) runs as a pre-pass before the crop/resize job."""
    from tests.test_ssd import SSD_AUG, random_boxes
    rng = np.random.default_rng(21)
    f = A.ParamFactory(SSD_AUG)
    states = A.seed_slots(5, 24)
    imgs, params = [], []
    for i in range(24):
        w, h = int(rng.integers(40, 400)), int(rng.integers(40, 400))
        imgs.append(A.synthetic_image(i, w, h, 3))
        st = states[i:i + 1].copy()
        params.append(f.make_ssd_params(st, w, h, 300, 300, random_boxes(rng, w, h, 3)))
    assert any(p.expand_ratio > 1 for p in params) and any(p.expand_ratio == 1 for p in params)
    for otype in ("uint8", "float32"):
        out = A.out_desc(channels=3, channel_major=True, dtype=otype, item_stride=3 * 300 * 300 * 4)
        _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "ssd " + otype)


@pytest.mark.parametrize("angle,rss", [(0, 0), (30, 0), (0, 200), (-90, 160)])
def test_expand_with_rotation_and_resize_short(ctx, angle, rss):
    """rotate -> expand -> resize_short -> crop (etl_image.cpp:146-170) with hand-built params;
    masks of the same params ignore the expand (etl_pixel_mask.cpp:65-90)."""
    rng = np.random.default_rng(angle + rss)
    imgs, masks, params = [], [], []
    for i in range(8):
        w, h = int(rng.integers(60, 300)), int(rng.integers(60, 300))
        imgs.append(A.synthetic_image(i, w, h, 3))
        masks.append(A.synthetic_image(50 + i, w, h, 1))
        ew, eh = int(w * 2.5), int(h * 2.5)
        ox, oy = int(rng.integers(0, ew - w + 1)), int(rng.integers(0, eh - h + 1))
        bw, bh = (ew, eh)
        if rss:
            s = rss / min(ew, eh)
            bw, bh = (rss, int(round(eh * s))) if ew <= eh else (int(round(ew * s)), rss)
        bw, bh = bw - 2, bh - 2  # margin for resize_short's rounding
        cw, ch = int(rng.integers(16, min(bw, w) + 1)), int(rng.integers(16, min(bh, h) + 1))
        params.append(A.aug_params(crop_x=int(rng.integers(0, bw - cw + 1)), crop_y=int(rng.integers(0, bh - ch + 1)),
                                   crop_w=cw, crop_h=ch, out_w=96, out_h=80, angle=angle, flip=i % 2,
                                   resize_short_size=rss, expand_ratio=2.5, expand_x=ox, expand_y=oy,
                                   expand_w=ew, expand_h=eh))
    out = A.out_desc(channels=3, channel_major=False, dtype="uint8", item_stride=3 * 96 * 80)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "expand")
    mparams = []
    for m, p in zip(masks, params):  # mask crops must fit the un-expanded (rotated) record
        q = A.aug_params(**{k: v for k, v in p.as_dict().items() if k != "lighting"})
        q.crop_x, q.crop_y = 0, 0
        q.crop_w, q.crop_h = min(p.crop_w, m.shape[1]), min(p.crop_h, m.shape[0])
        q.resize_short_size = 0
        mparams.append(q)
    mout = A.out_desc(channels=1, channel_major=True, dtype="uint8", item_stride=96 * 80)
    _assert_same(H.hip_records(ctx, masks, mparams, mout, mask=True),
                 H.oracle_records(masks, mparams, mout, mask=True), "expand mask")


def test_spec_bs_hue_primary_colours_and_greys(ctx):
    """Contrast pass 1's specialised loop on pixels at HSV sector boundaries (pure and mixed
    primaries: f = 0, two channels with the same weight) and on greys (s = 0, diff = 0)."""
    w, h = 240, 200
    img = np.zeros((h, w, 3), np.uint8)
    levels = np.arange(0, 256, 17, dtype=np.uint8)
    combos = [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (0, 1, 1), (1, 0, 1), (1, 1, 1), (2, 1, 0), (0, 2, 1)]
    for y in range(h):
        for x in range(w):
            c = combos[(x // 8) % len(combos)]
            v = int(levels[(y // 4) % len(levels)])
            img[y, x] = [min(255, v * k // 2 + (v if k else 0)) for k in c]
    params = [A.aug_params(crop_x=0, crop_y=0, crop_w=w, crop_h=h, out_w=224, out_h=224, flip=i & 1,
                           brightness=b, saturation=s, contrast=0.7, hue=hue)
              for i, (b, s, hue) in enumerate([(0.9, 1.5, 30), (0.6, 0.5, -60), (1.0, 2.0, 179), (0.8, 1.2, -1)])]
    imgs = [img] * len(params)
    out = A.out_desc(**MEAN_OUT)
    _assert_same(H.hip_records(ctx, imgs, params, out), H.oracle_records(imgs, params, out), "spec primaries")


@pytest.mark.parametrize("occ", ["1", "2"])
def test_split_kernel_opt_in(occ, monkeypatch):
    """augment_split (split_kernels.hip; AEON_HIP_SPLIT=1 -- measured slower than augment_tiles, DESIGN §4,
    kept opt-in): the C2 batch, both goldens' configuration (flip, non-multiple-of-4 crop) and the C5 image
    launch through the planner path, bit-exact against the oracle, with one and with two workgroups per CU."""
    monkeypatch.setenv("AEON_HIP_SPLIT", "1")
    monkeypatch.setenv("AEON_HIP_SPLIT_OCC", occ)
    monkeypatch.setenv("AEON_HIP_SPLIT_RPL", "1" if occ == "2" else "2")
    c = A.Context(0)
    try:
        n = 256
        imgs = _synthetic(n)
        params = H.draw_params(C.C2_AUG, [(256, 256)] * n, 224, 224, seed=3)
        out = A.out_desc(**MEAN_OUT)
        _assert_same(H.hip_records(c, imgs, params, out), H.oracle_records(imgs, params, out), "split C2")
        p = [A.aug_params(crop_x=50, crop_y=50, crop_w=171, crop_h=201, out_w=224, out_h=224, flip=f) for f in (0, 1)]
        two = _synthetic(2)
        _assert_same(H.hip_records(c, two, p, out), H.oracle_records(two, p, out), "split flip / odd crop")
        imgs5 = [A.synthetic_image(i, 640, 480, 3) for i in range(16)]
        params5 = H.draw_params(C.C5_AUG, [(640, 480)] * 16, 512, 512, seed=2)
        iout = C.out_desc_for(C.IMAGE_512, C.C5_AUG)
        _assert_same(H.hip_records(c, imgs5, params5, iout), H.oracle_records(imgs5, params5, iout), "split C5 images")
    finally:
        c.close()
