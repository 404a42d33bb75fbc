"""GPU parity of the one-launch contrast path (record_kernels.hip: the post-hue record held in the
lanes' registers, its table built from the exact sums, no u8 intermediate) against the oracle and
against the two-launch path (AEON_HIP_RECORDS=0), over what the kernel's schedule and register
rotation depend on: records per workgroup (1 .. 5 steps, a partial last round), output heights below
224 (fewer tiles per record than the rotation period), widths from 4 to 256, the fixed-point form of
every record (the FAST kernel) and records that need the generic form (diagonal / float
brightness-saturation: the GENERIC kernel), hue 0, contrast 1, lighting, padding and flips."""
import os

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu

MEAN = dict(channels=3, channel_major=True, bgr_to_rgb=True, dtype="float32", mean=C.MEAN, stddev=C.STDDEV)


@pytest.fixture(scope="module")
def ctxs():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    fused = A.Context(0)
    os.environ["AEON_HIP_RECORDS"] = "0"
    try:
        two = A.Context(0)  # the flag is read when a context is created
    finally:
        del os.environ["AEON_HIP_RECORDS"]
    yield fused, two
    fused.close()
    two.close()


def _check(ctxs, imgs, params, out_w, out_h, what):
    fused, two = ctxs
    out = A.out_desc(item_stride=3 * out_w * out_h * 4, **MEAN)
    a = H.hip_records(fused, imgs, params, out)
    b = H.hip_records(two, imgs, params, out)
    ref = H.oracle_records(imgs, params, out)
    for i in range(len(imgs)):
        assert np.array_equal(a[i], b[i]), f"{what}: record {i} fused != two-launch"
        if not np.array_equal(a[i], ref[i]):
            bad = np.argwhere(a[i] != ref[i])
            raise AssertionError(f"{what}: record {i}: {len(bad)} mismatches vs oracle, first {bad[0]}")


@pytest.mark.parametrize("n", [1, 5, 255, 300, 1100])
def test_records_c3_batch_sizes(ctxs, n):
    """1 .. 5 records per workgroup on the 256-CU grid, partial last rounds."""
    imgs = [A.synthetic_image(i, 256, 256, 3) for i in range(min(n, 64))]
    imgs = [imgs[i % len(imgs)] for i in range(n)]
    params = H.draw_params(C.C3_AUG, [(256, 256)] * n, 224, 224, seed=n)
    _check(ctxs, imgs, params, 224, 224, f"C3 n={n}")


@pytest.mark.parametrize("out_w,out_h", [(224, 200), (128, 96), (64, 32), (4, 17), (256, 224), (96, 224),
                                         (320, 96), (512, 48), (1024, 24)])
def test_records_output_sizes(ctxs, out_w, out_h):
    """Heights below 224 (fewer tiles than the register rotation), widths 4 .. 256."""
    rng = np.random.default_rng(out_w * 1000 + out_h)
    n = 40
    imgs = [A.synthetic_image(i, int(rng.integers(64, 400)), int(rng.integers(64, 400)), 3) for i in range(n)]
    params = H.draw_params(C.C3_AUG, [(im.shape[1], im.shape[0]) for im in imgs], out_w, out_h, seed=5)
    _check(ctxs, imgs, params, out_w, out_h, f"C3 {out_w}x{out_h}")


def test_records_mixed_photometric(ctxs):
    """hue 0, contrast 1, no lighting, saturation 1 (diagonal transform: the GENERIC kernel), a float
    transform (|M| >= 32), padding offsets, flips -- in one launch with fixed-point records."""
    rng = np.random.default_rng(17)
    imgs, params = [], []
    for i in range(48):
        w, h = int(rng.integers(150, 420)), int(rng.integers(150, 420))
        imgs.append(A.synthetic_image(1000 + i, w, h, 3))
        cw, ch = int(rng.integers(60, w)), int(rng.integers(60, h))
        kw = dict(crop_x=int(rng.integers(0, w - cw + 1)), crop_y=int(rng.integers(0, h - ch + 1)), crop_w=cw,
                  crop_h=ch, out_w=224, out_h=224, flip=int(i % 2), contrast=float(rng.uniform(0.5, 1.0)),
                  brightness=float(rng.uniform(0.5, 1.0)), saturation=float(rng.uniform(0.5, 2.0)),
                  hue=int(rng.integers(-18, 19)))
        if i % 5 == 0:
            kw["hue"] = 0
        if i % 7 == 0:
            kw["contrast"] = 1.0
        if i % 3 == 0:
            kw["lighting"] = [float(x) for x in rng.normal(0, 0.1, 3)]
            kw["color_noise_std"] = 0.1
        if i == 11:
            kw["saturation"] = 1.0  # diagonal cv::transform
        if i == 13:
            kw["brightness"], kw["saturation"] = 40.0, 1.5  # float cv::transform
        if i % 4 == 1:
            kw.update(padding=4, pad_off_x=int(rng.integers(0, 9)), pad_off_y=int(rng.integers(0, 9)))
        params.append(A.aug_params(**kw))
    _check(ctxs, imgs, params, 224, 224, "mixed photometric")
    # and the same records without the generic ones: the FAST kernel over hue 0 / contrast 1 / padding
    keep = [i for i in range(48) if i not in (11, 13)]
    _check(ctxs, [imgs[i] for i in keep], [params[i] for i in keep], 224, 224, "fast kernel mix")


def test_records_real_image_and_rerun(ctxs, golden):
    """aeon's own record under C3 (natural-image hue tables), twice: bit-identical."""
    fused, _ = ctxs
    imgs = [golden["img"]] * 300
    params = H.draw_params(C.C3_AUG, [(480, 360)] * 300, 224, 224, seed=21)
    out = A.out_desc(item_stride=3 * 224 * 224 * 4, **MEAN)
    r1 = H.hip_records(fused, imgs, params, out)
    r2 = H.hip_records(fused, imgs, params, out)
    assert all(np.array_equal(a, b) for a, b in zip(r1, r2))
    ref = H.oracle_records(imgs[:40], params[:40], out)
    assert all(np.array_equal(a, b) for a, b in zip(r1[:40], ref))

