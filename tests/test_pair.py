"""aeon_hip_augment_pair_batch: provider::image + provider::pixelmask of the same records in one
call (aeon src/provider.cpp:109-119, 365-393: one params set per record for both).  By default one
job-table upload serves both and the masks' gather pass is a launch of its own; with
AEON_HIP_FUSE_MASKS=1 the masks' NEAREST row blocks run inside the image tile launch
(augment_kernels.hip mask_blocks).  Every byte must equal the two separate calls' and the oracle's in
both forms, and the fused form must really be one launch.  The module's context is the fused form."""
import os

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _ctx(fuse=True):
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    old = os.environ.get("AEON_HIP_FUSE_MASKS")
    os.environ["AEON_HIP_FUSE_MASKS"] = "1" if fuse else "0"
    try:
        return A.Context(0)
    finally:
        if old is None:
            del os.environ["AEON_HIP_FUSE_MASKS"]
        else:
            os.environ["AEON_HIP_FUSE_MASKS"] = old


@pytest.fixture(scope="module")
def ctx():
    c = _ctx(True)
    yield c
    c.close()


def _items(host, params, out):
    res = []
    for i, p in enumerate(params):
        cn = out.channels
        shape = (cn, p.out_h, p.out_w) if out.channel_major else (p.out_h, p.out_w, cn)
        dt = A.NP_DTYPE[out.dtype]
        nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
        res.append(host[i * out.item_stride: i * out.item_stride + nbytes].view(dt).reshape(shape).copy())
    return res


def _pair(ctx, imgs, masks, params, iout, mout, calls=1):
    """One pair call (or `calls` in a row into fresh buffers); returns ([images], [masks]) of the last,
    and the launches the context timed per call."""
    import torch
    ia, idescs = A.pack_images(imgs)
    ma, mdescs = A.pack_images(masks)
    isrc, msrc = torch.from_numpy(ia).to("cuda"), torch.from_numpy(ma).to("cuda")
    n = len(imgs)
    stream = torch.cuda.current_stream().cuda_stream
    ctx.kernel_times()
    ctx.set_timing(1)
    for _ in range(calls):
        idst = torch.full((n * iout.item_stride,), 0xAB, dtype=torch.uint8, device="cuda")
        mdst = torch.full((n * mout.item_stride,), 0xCD, dtype=torch.uint8, device="cuda")
        ctx.pair_batch(idescs, isrc.data_ptr(), mdescs, msrc.data_ptr(), params, iout, idst.data_ptr(), mout,
                       mdst.data_ptr(), stream)
    ctx.synchronize(stream)
    launches = ctx.kernel_times()["augment"][2] / calls
    ctx.set_timing(False)
    return _items(idst.cpu().numpy(), params, iout), _items(mdst.cpu().numpy(), params, mout), launches


def _same(a, b, what):
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert x.shape == y.shape, (what, i)
        if not np.array_equal(x, y):
            bad = np.argwhere(x != y)
            raise AssertionError(f"{what}: record {i} differs at {len(bad)} elements, first {bad[0].tolist()}")


def _c5(n, seed):
    rng = np.random.default_rng(seed)
    imgs = [A.synthetic_image(i, 640, 480, 3) for i in range(n)]
    masks = [rng.integers(0, 21, (480, 640), dtype=np.uint8) for _ in range(n)]
    params = H.draw_params(C.C5_AUG, [(640, 480)] * n, 512, 512, seed=seed)
    return imgs, masks, params, C.out_desc_for(C.IMAGE_512, C.C5_AUG), C.out_desc_for(C.MASK_512, C.C5_AUG)


@pytest.mark.parametrize("fused", [True, False])
def test_pair_c5_full_batch(ctx, fused):
    """BASELINE C5 at its size (128 pairs, 640x480 -> 512x512), three calls in a row (the fused form's
    mask-block counter resets itself): one launch per call fused, two (tiles + gather) by default;
    every record of both outputs equal to the oracle."""
    imgs, masks, params, iout, mout = _c5(128, 5)
    c = ctx if fused else _ctx(False)
    try:
        hi, hm, launches = _pair(c, imgs, masks, params, iout, mout, calls=3)
    finally:
        if not fused:
            c.close()
    assert launches == (1 if fused else 2), f"{launches} timed launches per pair call"
    _same(hi, H.oracle_records(imgs, params, iout), "C5 pair image")
    _same(hm, H.oracle_records(masks, params, mout, mask=True), "C5 pair mask")


def test_pair_equals_separate_calls(ctx):
    """The fused call against the same context's two separate calls and an unfused context."""
    imgs, masks, params, iout, mout = _c5(40, 9)
    hi, hm, _ = _pair(ctx, imgs, masks, params, iout, mout)
    si = H.hip_records(ctx, imgs, params, iout)
    sm = H.hip_records(ctx, masks, params, mout, mask=True)
    _same(hi, si, "pair vs augment_batch")
    _same(hm, sm, "pair vs mask_batch")
    c2 = _ctx(False)
    try:
        ui, um, launches = _pair(c2, imgs, masks, params, iout, mout)
    finally:
        c2.close()
    assert launches == 2, launches
    _same(hi, ui, "fused vs unfused image")
    _same(hm, um, "fused vs unfused mask")


@pytest.mark.parametrize("case", ["ragged_rows", "downscale", "narrow", "one", "uint8_image"])
def test_pair_edge_cases(ctx, case):
    """Output heights that are not a multiple of the 64-row blocks, horizontal downscales beyond 4/3
    (the per-element gather), widths that leave rows unaligned to 16 bytes, a single pair, and a
    uint8 HWC image output next to the mask -- all against the oracle."""
    rng = np.random.default_rng(sum(map(ord, case)))
    aug = {"type": "image", "center": False, "scale": [0.3, 1.0], "flip_enable": True}
    ow, oh, n, src = 200, 150, 24, (320, 240)
    img_etl = {"type": "image", "channels": 3, "output_type": "float", "channel_major": True}
    if case == "downscale":
        ow, oh, src = 96, 80, (400, 300)
        aug = dict(aug, scale=[0.9, 1.0])
    elif case == "narrow":
        ow, oh = 52, 70
    elif case == "one":
        n = 1
    elif case == "uint8_image":
        img_etl = {"type": "image", "channels": 3, "output_type": "uint8_t", "channel_major": False}
    img_etl = dict(img_etl, width=ow, height=oh)
    mask_etl = {"type": "pixelmask", "width": ow, "height": oh, "channels": 1, "output_type": "uint8_t"}
    sizes = [(src[0] - 8 * (i % 5), src[1] - 6 * (i % 3)) for i in range(n)]
    imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
    masks = [rng.integers(0, 256, (h, w), dtype=np.uint8) for (w, h) in sizes]
    params = H.draw_params(aug, sizes, ow, oh, seed=11)
    iout, mout = C.out_desc_for(img_etl, aug), C.out_desc_for(mask_etl, aug)
    hi, hm, launches = _pair(ctx, imgs, masks, params, iout, mout)
    _same(hi, H.oracle_records(imgs, params, iout), f"{case} image")
    _same(hm, H.oracle_records(masks, params, mout, mask=True), f"{case} mask")


def test_pair_unfusable_masks_fall_back(ctx):
    """Masks the fused launch does not take (float32 mask items) go as the two calls, same bytes."""
    imgs, masks, params, iout, _ = _c5(8, 13)
    mout = C.out_desc_for(dict(C.MASK_512, output_type="float"), C.C5_AUG)
    hi, hm, launches = _pair(ctx, imgs, masks, params, iout, mout)
    assert launches == 2, launches
    _same(hi, H.oracle_records(imgs, params, iout), "fallback image")
    _same(hm, H.oracle_records(masks, params, mout, mask=True), "fallback mask")


@pytest.mark.parametrize("vram", [True, False])
def test_ring_reuse_changing_params(vram):
    """20 calls in a row on one context (more than its 16 ring slots) with different params each
    time, C2 direct calls and C5 pair calls interleaved, outputs checked per call: the job tables the
    host writes into HBM through the BAR (or, AEON_HIP_VRAM_JOBS=0, pinned host tables) are never read
    stale when a slot comes round again."""
    import torch
    old = os.environ.get("AEON_HIP_VRAM_JOBS")
    os.environ["AEON_HIP_VRAM_JOBS"] = "1" if vram else "0"
    try:
        c = A.Context(0)
    finally:
        if old is None:
            del os.environ["AEON_HIP_VRAM_JOBS"]
        else:
            os.environ["AEON_HIP_VRAM_JOBS"] = old
    try:
        n = 12
        imgs = [A.synthetic_image(i, 256, 256, 3) for i in range(n)]
        out224 = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
        arena, descs = A.pack_images(imgs)
        src = torch.from_numpy(arena).to("cuda")
        stream = torch.cuda.current_stream().cuda_stream
        c5 = _c5(6, 21)
        pending = []
        for call in range(20):
            params = H.draw_params(C.C2_AUG, [(256, 256)] * n, 224, 224, seed=100 + call)
            dst = torch.empty(n * out224.item_stride, dtype=torch.uint8, device="cuda")
            c.augment_batch(descs, src.data_ptr(), params, out224, dst.data_ptr(), stream)
            pending.append((params, dst))
            if call % 5 == 4:  # a pair call between them (planner path: its table in the next slot)
                hi, hm, _ = _pair(c, *c5)
                _same(hm, H.oracle_records(c5[1], c5[2], c5[4], mask=True), f"pair mask at call {call}")
        c.synchronize(stream)
        for call, (params, dst) in enumerate(pending):
            got = _items(dst.cpu().numpy(), params, out224)
            _same(got, H.oracle_records(imgs, params, out224), f"C2 call {call}")
    finally:
        c.close()


@pytest.mark.parametrize("n", [3000, 5000])
def test_large_tables_take_the_other_transports(n):
    """Calls whose job table is past the direct path's per-tile fetch budget (3,000 records: the
    planner path with its table in HBM) and past the HBM table size (5,000 records, 1.28 MB: the SDMA
    upload), tiny records so the oracle stays quick -- every record against it."""
    import torch
    c = A.Context(0)
    try:
        rng = np.random.default_rng(n)
        sizes = [(40 + int(rng.integers(0, 9)), 36 + int(rng.integers(0, 9))) for _ in range(n)]
        imgs = [A.synthetic_image(i, w, h, 3) for i, (w, h) in enumerate(sizes)]
        aug = {"type": "image", "center": False, "scale": [0.6, 1.0], "flip_enable": True}
        etl = {"type": "image", "width": 32, "height": 32, "channels": 3, "output_type": "float",
               "channel_major": True, "bgr_to_rgb": True}
        out = C.out_desc_for(etl, aug)
        params = H.draw_params(aug, sizes, 32, 32, seed=n)
        got = H.hip_records(c, imgs, params, out)
        _same(got, H.oracle_records(imgs, params, out), f"{n} records")
    finally:
        c.close()
