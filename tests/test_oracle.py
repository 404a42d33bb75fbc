"""CPU: the oracle against aeon's golden vectors and known-answer tests.

Pins the oracle: bit-exact on augment_output_linear_{train,eval}.bin and on
the KATs of test/test_image.cpp / test_pixel_mask.cpp / test_util.cpp restated here.
"""
import numpy as np
import pytest

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def test_golden_train(oracle, golden):
    O = oracle
    p = O.params(crop_x=50, crop_y=50, crop_w=171, crop_h=201, out_w=224, out_h=224, flip=1)
    out = O.augment_record(golden["img"], p, O.load_config(3, True, True, "float32", MEAN, STD))
    assert np.array_equal(out, golden["train"])


def test_golden_eval(oracle, golden):
    O = oracle
    f = O.Factory(O.aug_config(scale_min=0.875, scale_max=0.875, resize_short_size=256))
    st = np.array([1], np.uint32)
    p = f.make_params(st, 480, 360, 224, 224)
    assert (p.crop_x, p.crop_y, p.crop_w, p.crop_h) == (58, 16, 224, 224)
    out = O.augment_record(golden["img"], p, O.load_config(3, True, True, "float32", MEAN, STD))
    assert np.array_equal(out, golden["eval"])


def _bands(vals):
    img = np.zeros((384, 512, 3), np.uint8)
    for k, v in enumerate(vals):
        img[128 * k:128 * (k + 1)] = v
    return img


@pytest.mark.parametrize("c,expect", [(1.0, (0, 127, 255)), (0.5, (64, 127, 191)), (0.1, (115, 127, 140))])
def test_kat_contrast(oracle, c, expect):
    """test/test_image.cpp:1367-1418 photometric.contrast"""
    out = oracle.cbsjitter(_bands((0, 127, 255)), contrast=c)
    for k, v in enumerate(expect):
        assert (out[128 * k:128 * (k + 1)] == v).all()


@pytest.mark.parametrize("b,expect", [(1.0, (0, 127, 255)), (0.5, (0, 64, 128)), (0.1, (0, 13, 26)),
                                      (1.5, (0, 190, 255))])
def test_kat_brightness(oracle, b, expect):
    """test/test_image.cpp:1420-1480 photometric.brightness"""
    out = oracle.cbsjitter(_bands((0, 127, 255)), brightness=b)
    for k, v in enumerate(expect):
        assert (out[128 * k:128 * (k + 1)] == v).all()


def _indexed(rows, cols):
    """generate_indexed_image (test/test_image.cpp:42-57): b=col, g=row, r=0."""
    img = np.zeros((rows, cols, 3), np.uint8)
    img[:, :, 0] = np.arange(cols, dtype=np.uint8)[None, :]
    img[:, :, 1] = np.arange(rows, dtype=np.uint8)[:, None]
    return img


def test_kat_crop(oracle):
    """image.transform_crop (test/test_image.cpp:462-493)"""
    out = oracle.transform_image(_indexed(256, 256), oracle.params(crop_x=100, crop_y=150, crop_w=20,
                                                                   crop_h=30, out_w=20, out_h=30))
    assert out.shape == (30, 20, 3)
    assert tuple(out[0, 0, :2]) == (100, 150)
    assert tuple(out[0, 19, :2]) == (119, 150)
    assert tuple(out[29, 0, :2]) == (100, 179)


def test_kat_flip(oracle):
    """image.transform_flip (test/test_image.cpp:564-595)"""
    out = oracle.transform_image(_indexed(256, 256), oracle.params(crop_x=100, crop_y=150, crop_w=20,
                                                                   crop_h=20, out_w=20, out_h=20, flip=1))
    assert tuple(out[0, 0, :2]) == (119, 150)
    assert tuple(out[0, 19, :2]) == (100, 150)
    assert tuple(out[19, 0, :2]) == (119, 169)


@pytest.mark.parametrize("w,h,pad,ox,oy", [(32, 32, 5, 2, 8), (32, 32, 5, 5, 5), (32, 32, 4, 0, 0),
                                           (30, 30, 5, 10, 10), (30, 30, 0, 0, 0), (1, 1, 10, 0, 20),
                                           (2, 2, 10, 10, 10)])
def test_kat_padding(oracle, w, h, pad, ox, oy):
    """image.transform_padding (test/test_image.cpp:597-684)"""
    out = oracle.transform_image(_indexed(h, w), oracle.params(crop_x=0, crop_y=0, crop_w=w, crop_h=h,
                                                               out_w=w, out_h=h, padding=pad,
                                                               pad_off_x=ox, pad_off_y=oy))
    for row in range(h + 2 * pad):
        for col in range(w + 2 * pad):
            if row < oy or col < ox or row >= oy + h or col >= ox + w:
                continue
            px = out[row - oy, col - ox]
            if col < pad or col >= w + pad or row < pad or row >= h + pad:
                assert tuple(px) == (0, 0, 0)
            else:
                assert tuple(px) == (col - pad, row - pad, 0)


def test_kat_mask_nearest(oracle):
    """test/test_pixel_mask.cpp:76-236: NEAREST never invents values."""
    rng = np.random.default_rng(0)
    m = (rng.integers(0, 2, (300, 400)) * 255).astype(np.uint8)
    p = oracle.params(crop_x=13, crop_y=17, crop_w=333, crop_h=250, out_w=512, out_h=512, flip=1)
    out = oracle.transform_mask(m, p)
    assert set(np.unique(out)) <= {0, 255}


def test_kat_hue_zero_and_full_turn(oracle):
    img = np.random.default_rng(1).integers(0, 256, (16, 16, 3), dtype=np.uint8)
    assert np.array_equal(oracle.cbsjitter(img, hue=0), img)
    # 180 and 360 are both full turns of OpenCV's 8-bit hue: the same HSV8 round trip
    assert np.array_equal(oracle.cbsjitter(img, hue=180), oracle.cbsjitter(img, hue=360))


def test_resize_identity_and_area2x(oracle):
    img = np.random.default_rng(2).integers(0, 256, (64, 48, 3), dtype=np.uint8)
    assert np.array_equal(oracle.resize_linear(img, 48, 64), img)
    half = oracle.resize_linear(img, 24, 32)
    i = img.astype(np.int32)
    ref = (i[0::2, 0::2] + i[0::2, 1::2] + i[1::2, 0::2] + i[1::2, 1::2] + 2) >> 2
    assert np.array_equal(half, ref.astype(np.uint8))


def test_standardize_values(oracle):
    # the f64-per-op formula pinned by the goldens, spot values
    v = oracle.lib().orc_standardize_value(255, 0.485, 0.229)
    assert abs(v - (1.0 - 0.485) / 0.229) < 1e-6


@pytest.mark.parametrize("esize,dtype", [(1, np.uint8), (2, np.uint16), (4, np.uint32), (8, np.uint64)])
def test_transpose_restatement(oracle, esize, dtype):
    # transpose_regular (src/buffer_batch.cpp:186-200): dest[c*rows + r] = src[r*cols + c]
    rows, cols = 5, 9
    m = np.arange(rows * cols, dtype=dtype).reshape(rows, cols)
    out = oracle.transpose(m, rows, cols, esize).view(dtype).reshape(cols, rows)
    assert np.array_equal(out, m.T)
    with pytest.raises(RuntimeError, match="unsupported datatype"):
        oracle.transpose(np.zeros(15, np.uint8), 5, 1, 3)


# ---- image::rotate (src/image.cpp:53-75; OpenCV 2.4 warpAffine) -----------------------------
@pytest.mark.parametrize("interp", [True, False])
def test_rotate_exact_quarter_turns(oracle, interp):
    # about the integer centre of an odd square, 180 degrees is an exact double flip and +90 is
    # OpenCV's documented counter-clockwise quarter turn
    img = (np.arange(9 * 9 * 3) % 251).astype(np.uint8).reshape(9, 9, 3)
    assert np.array_equal(oracle.rotate(img, 180, interp), img[::-1, ::-1])
    assert np.array_equal(oracle.rotate(img, 90, interp), np.rot90(img, 1))
    assert np.array_equal(oracle.rotate(img, 0, interp), img)


def test_rotate_mask_nearest_keeps_classes(oracle):
    # test/test_pixel_mask.cpp:130-155 (pixel_mask rotate 45): nearest rotation invents no values
    m = np.zeros((64, 80), np.uint8)
    m[10:30, 5:40] = 7
    m[35:60, 20:70] = 200
    r = oracle.rotate(m, 45, False)
    assert set(np.unique(r)) <= {0, 7, 200}
    assert len(np.unique(oracle.rotate(m, 45, True))) > 3  # bilinear blends edges
