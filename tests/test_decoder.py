"""GPU: the decode stage (provider_factory + batch_decoder through the C ABI) against the oracle,
with aeon's deterministic mode: slot engines seeded from minstd_rand0(random_seed + node_id)."""
import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu


def _records(n, seed=0, mask=False):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        w, h = int(rng.integers(200, 700)), int(rng.integers(200, 700))
        img = A.synthetic_image(i + 1000 * seed, w, h, 3)
        if mask:
            m = ((A.synthetic_image(50000 + i, w, h, 1) > 100) * 255).astype(np.uint8)
            recs.append((img, m))
        else:
            recs.append((img,))
    return recs


def _oracle(recs, params, etl, aug, mask_k=None):
    outs = []
    for k, e in enumerate(etl):
        od = C.out_desc_for(e, aug)
        outs.append(np.stack(H.oracle_records([r[k] for r in recs], params, od, mask=(k == mask_k))))
    return outs


def test_decoder_c3_two_windows():
    cfg = dict(batch_size=8, random_seed=5, etl=[C.IMAGE_224], augmentation=[C.C3_AUG])
    d = A.Decoder(cfg)
    f = A.ParamFactory(C.C3_AUG)  # the checker's params: same slots, same record order
    states = A.seed_slots(5, 8)
    for window in range(2):
        recs = _records(8, seed=window)
        params = [f.make_params(states[i:i + 1], r[0].shape[1], r[0].shape[0], 224, 224)
                  for i, r in enumerate(recs)]
        (out,) = d.decode(recs)
        (ref,) = _oracle(recs, params, [C.IMAGE_224], C.C3_AUG)
        assert np.array_equal(out, ref), f"window {window}"


def test_decoder_c5_image_and_mask():
    cfg = dict(batch_size=6, random_seed=3, node_id=1, node_count=2, etl=[C.IMAGE_512, C.MASK_512],
               augmentation=[C.C5_AUG])
    d = A.Decoder(cfg)
    recs = _records(6, seed=2, mask=True)
    params = H.draw_params(C.C5_AUG, [(r[0].shape[1], r[0].shape[0]) for r in recs], 512, 512, seed=3 + 1)
    img, msk = d.decode(recs)
    ref_img, ref_msk = _oracle(recs, params, [C.IMAGE_512, C.MASK_512], C.C5_AUG, mask_k=1)
    assert np.array_equal(img, ref_img)
    assert np.array_equal(msk, ref_msk)


def test_decoder_empty_record_raises():
    d = A.Decoder(dict(batch_size=2, etl=[C.IMAGE_224], augmentation=[C.C2_AUG]))
    with pytest.raises(A.AeonHipError) as e:
        d.decode([(np.zeros((0, 0, 3), np.uint8),)])
    assert "size 0" in str(e.value)


def test_decoder_batch_major_false_transposes_each_batch():
    # batch_major=false (loader.hpp:63): each batch arrives as [element][record]
    # (batch_iterator.cpp:125-136 -> transpose_buf, buffer_batch.cpp:251-280)
    import oracle as O
    cfg = dict(batch_size=4, random_seed=9, etl=[C.IMAGE_224], augmentation=[C.C2_AUG])
    recs = _records(8, seed=4)
    (ref,) = A.Decoder(cfg).decode(recs)
    (out,) = A.Decoder(dict(cfg, batch_major=False)).decode(recs)
    item = ref[0].nbytes
    raw = ref.reshape(-1).view(np.uint8)
    got = out.reshape(-1).view(np.uint8)
    for b in range(2):
        blk = raw[b * 4 * item:(b + 1) * 4 * item]
        assert np.array_equal(got[b * 4 * item:(b + 1) * 4 * item], O.transpose(blk, 4, item // 4, 4)), b


def test_decoder_batch_major_false_needs_whole_batches():
    cfg = dict(batch_size=4, random_seed=9, batch_major=False, etl=[C.IMAGE_224], augmentation=[C.C2_AUG])
    with pytest.raises(A.AeonHipError, match="whole batches"):
        A.Decoder(cfg).decode(_records(3, seed=4))


def test_decoder_fixed_aspect_ratio_uint8():
    """provider::image with the augmentation's fixed_aspect_ratio (image::loader ctor,
    provider.cpp:145-158): each record scaled to fit and written at the top-left of its zeroed
    256x256 uint8 canvas."""
    aug = {"type": "image", "fixed_aspect_ratio": True, "crop_enable": False, "flip_enable": True}
    etl = {"type": "image", "height": 256, "width": 256, "channels": 3, "output_type": "uint8_t",
           "channel_major": True, "bgr_to_rgb": True}
    d = A.Decoder(dict(batch_size=6, random_seed=9, etl=[etl], augmentation=[aug]))
    recs = _records(6, seed=4)
    params = H.draw_params(aug, [(r[0].shape[1], r[0].shape[0]) for r in recs], 256, 256, seed=9)
    (out,) = d.decode(recs)
    od = C.out_desc_for(etl, aug)
    ref = np.stack([H.place_canvas(r, od) for r in H.oracle_records([r[0] for r in recs], params, od)])
    assert np.array_equal(out, ref)


def _jpeg_files():
    import os
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "jpeg_fixtures.npz"))
    names = sorted({k.rsplit(".", 1)[0] for k in fx.files})
    return [fx[n + ".jpg"].tobytes() for n in names]


def test_decoder_encoded_jpeg_records_c1():
    """provider::image::provide end to end from encoded records (image::extractor::extract ->
    transform -> load): JPEG files through the JPEG stage and the C1 eval transform, against the
    oracle's decode + transform + load of the same files (the golden img_2112_70.jpg among them)."""
    import oracle as O
    files = _jpeg_files()
    files = [f for f in files if min(O.jpeg_info(f)[:2]) >= 8]  # resize_short of the smallest is degenerate
    cfg = dict(batch_size=len(files), random_seed=7, etl=[C.IMAGE_224], augmentation=[C.C1_AUG])
    (out,) = A.Decoder(cfg).decode([(f,) for f in files])
    dec = [O.jpeg_decode(f, 3) for f in files]
    params = H.draw_params(C.C1_AUG, [(d.shape[1], d.shape[0]) for d in dec], 224, 224, seed=7)
    (ref,) = _oracle([(d,) for d in dec], params, [C.IMAGE_224], C.C1_AUG)
    assert np.array_equal(out, ref)


def test_decoder_encoded_and_decoded_elements_mix():
    """An encoded JPEG image element next to a decoded pixel-mask element (C5 shape): the mask
    shares the image's params, and the JPEG record equals its pre-decoded twin."""
    import oracle as O
    files = [f for f in _jpeg_files() if min(O.jpeg_info(f)[:2]) >= 32][:6]
    dec = [O.jpeg_decode(f, 3) for f in files]
    masks = [((A.synthetic_image(70 + i, d.shape[1], d.shape[0], 1) > 127) * 255).astype(np.uint8)
             for i, d in enumerate(dec)]
    cfg = dict(batch_size=len(files), random_seed=3, etl=[C.IMAGE_512, C.MASK_512], augmentation=[C.C5_AUG])
    img_a, msk_a = A.Decoder(cfg).decode([(f, m) for f, m in zip(files, masks)])
    img_b, msk_b = A.Decoder(cfg).decode([(d, m) for d, m in zip(dec, masks)])
    assert np.array_equal(img_a, img_b) and np.array_equal(msk_a, msk_b), (
        _diff_report(img_a, img_b), int((msk_a != msk_b).sum()))


def test_decoder_submit_wait_double_buffered():
    """aeon_decoder_submit / wait: two windows in flight on the decoder's streams (async_manager's
    two containers) give exactly the synchronous decode's outputs, window by window (windows 1 and 3
    as records marshalled once, Decoder.encoded); a third submit before a wait is refused."""
    import torch
    files = _jpeg_files()
    files = [f for f in files if min(A.jpeg_info(f)[:2]) >= 8]
    cfg = dict(batch_size=len(files), random_seed=11, etl=[C.IMAGE_224], augmentation=[C.C2_AUG])
    windows = [[(files[(i + w) % len(files)],) for i in range(len(files))] for w in range(4)]
    sync = A.Decoder(cfg)
    want = [sync.decode(win)[0] for win in windows]
    d = A.Decoder(cfg)
    windows = [d.encoded(win) if w % 2 else win for w, win in enumerate(windows)]
    item = 3 * 224 * 224 * 4
    bufs = [torch.empty(len(files) * item, dtype=torch.uint8).pin_memory() for _ in range(2)]
    got = []
    d.submit(windows[0], [bufs[0].data_ptr()])
    d.submit(windows[1], [bufs[1].data_ptr()])
    with pytest.raises(A.AeonHipError, match="in flight"):
        d.submit(windows[2], [bufs[0].data_ptr()])
    for w in range(4):
        d.wait()
        got.append(bufs[w % 2].numpy().view(np.float32).reshape(want[w].shape).copy())
        if w + 2 < 4:
            d.submit(windows[w + 2], [bufs[w % 2].data_ptr()])
    for w in range(4):
        assert np.array_equal(got[w], want[w]), w


def test_decoder_png_image_and_mask():
    """Encoded PNG records (image::extractor / pixel_mask::extractor over cv::imdecode, decoded on
    the host pool while staging): an RGB image and gray / palette / 16-bit gray masks, against the
    oracle's PNG decode (oracle/png_oracle.py) and transforms."""
    import io

    from PIL import Image

    from oracle import png_oracle as PO

    def png_of(arr, mode=None, palette=None):
        im = Image.fromarray(arr, mode) if mode else Image.fromarray(arr)
        if palette is not None:
            im.putpalette(palette)
        buf = io.BytesIO()
        im.save(buf, "PNG")
        return buf.getvalue()

    rng = np.random.default_rng(11)
    recs, decoded = [], []
    for i in range(6):
        w, h = int(rng.integers(200, 360)), int(rng.integers(160, 300))
        img = A.synthetic_image(700 + i, w, h, 3)
        cls = (A.synthetic_image(900 + i, w, h, 1) % 5).astype(np.uint8)
        if i % 3 == 0:
            mpng = png_of(cls * 40)
        elif i % 3 == 1:
            mpng = png_of(cls, "P", [v for c in range(5) for v in (c * 30, c * 50, 255 - c * 40)])
        else:
            mpng = png_of((cls.astype(np.uint16) * 97 + (i * 13)).astype(np.uint16))
        recs.append((png_of(img[:, :, ::-1].copy()), mpng))
        decoded.append((PO.decode(recs[-1][0], PO.BGR8), PO.decode(mpng, PO.ANYDEPTH)))
    assert np.array_equal(decoded[0][0], A.decode_png(recs[0][0]))
    cfg = dict(batch_size=6, random_seed=4, etl=[C.IMAGE_512, C.MASK_512], augmentation=[C.C5_AUG])
    d = A.Decoder(cfg)
    img, msk = d.decode(recs)
    params = H.draw_params(C.C5_AUG, [(r[0].shape[1], r[0].shape[0]) for r in decoded], 512, 512, seed=4)
    iod = C.out_desc_for(C.IMAGE_512, C.C5_AUG)
    ref_img = np.stack(H.oracle_records([r[0] for r in decoded], params, iod))
    assert np.array_equal(img, ref_img)
    mod = C.out_desc_for(C.MASK_512, C.C5_AUG)
    for i, (r, p) in enumerate(zip(decoded, params)):
        m = r[1]
        if m.dtype == np.uint16:  # saturate_cast<uchar> of the 16-bit NEAREST result
            lo = H.oracle_records([(m & 0xff).astype(np.uint8)], [p], mod, mask=True)[0]
            hi = H.oracle_records([(m >> 8).astype(np.uint8)], [p], mod, mask=True)[0]
            want = np.minimum(hi.astype(np.uint32) * 256 + lo, 255).astype(np.uint8)
        else:
            want = H.oracle_records([m], [p], mod, mask=True)[0]
        assert np.array_equal(msk[i], want.reshape(msk[i].shape)), i


def _diff_report(want, got):
    """Where two outputs differ (for an assertion message): element offsets, 128-byte lines touched,
    the first wrong values next to the right ones, and where the wrong values occur in the right output."""
    dt = {4: np.float32, 2: np.uint16}.get(want.dtype.itemsize, np.uint8)
    a, b = want.reshape(-1).view(dt), got.reshape(-1).view(dt)
    ut = {4: np.uint32, 2: np.uint16}.get(want.dtype.itemsize, np.uint8)
    d = np.nonzero(a.view(ut) != b.view(ut))[0]
    if not len(d):
        return "equal"
    es = a.itemsize
    lines = np.unique(d * es // 128)
    where = [np.nonzero(b.view(ut) == a.view(ut)[i])[0][:3].tolist() for i in d[:6]]
    return (f"{len(d)} elements differ in [{d[0]}, {d[-1]}] ({d[0] * es:#x}..{d[-1] * es + es:#x}), {len(lines)} "
            f"lines of 128 B ({lines[0]}..{lines[-1]}); first wrong {a[d[:6]].tolist()} right {b[d[:6]].tolist()}; "
            f"wrong hex {[hex(int(x)) for x in a.view(ut)[d[:6]]]}; the wrong values at these offsets of the right "
            f"output: {where}")


def _decode_pinned(d, recs):
    """One window through submit/wait into pinned host buffers: the kernels store there directly
    (zero-copy host outputs)."""
    import torch
    bufs = [torch.full((len(recs) * o["item_bytes"],), 0xCD, dtype=torch.uint8).pin_memory() for o in d.outputs]
    d.submit(recs, [b.data_ptr() for b in bufs])
    d.wait()
    return [b.numpy().view(o["dtype"]).reshape((len(recs),) + o["shape"]).copy() for b, o in zip(bufs, d.outputs)]


@pytest.mark.parametrize("case", ["c5", "batch_major_false", "fixed_aspect_ratio"])
def test_decoder_zero_copy_outputs_match_staged(case):
    """Pinned host outputs are written by the kernels themselves (zero_copy_view, host.cpp); pageable
    ones are staged on the device and copied: the same bytes, including the transposed
    (batch_major=false) layout and fixed_aspect_ratio's zeroed canvases."""
    if case == "c5":
        cfg = dict(batch_size=6, random_seed=3, etl=[C.IMAGE_512, C.MASK_512], augmentation=[C.C5_AUG])
        recs = _records(6, seed=2, mask=True)
    elif case == "batch_major_false":
        cfg = dict(batch_size=4, random_seed=9, batch_major=False, etl=[C.IMAGE_224], augmentation=[C.C3_AUG])
        recs = _records(8, seed=4)
    else:
        aug = {"type": "image", "fixed_aspect_ratio": True, "crop_enable": False, "flip_enable": True}
        etl = {"type": "image", "height": 256, "width": 256, "channels": 3, "output_type": "float",
               "channel_major": True, "bgr_to_rgb": True}
        cfg = dict(batch_size=6, random_seed=9, etl=[etl], augmentation=[aug])
        recs = _records(6, seed=4)
    want = A.Decoder(cfg).decode(recs)
    got = _decode_pinned(A.Decoder(cfg), recs)
    for w, g in zip(want, got):
        assert w.dtype == g.dtype, case
        assert np.array_equal(w.view(np.uint8), g.view(np.uint8)), (case, _diff_report(w, g))


def test_decoder_after_contexts_come_and_go():
    """Contexts created and destroyed before a decode (each with its HBM job tables): the later
    device allocations still get every kernel write.  Freed uncached table blocks once came back as
    ordinary device memory that lost 128-byte lines of a contrast record's output (zeros); the tables
    are pooled for the process since (stage.cpp free_vram)."""
    od = C.out_desc_for(C.IMAGE_224, C.C3_AUG)
    f = A.ParamFactory(C.C3_AUG)
    eng = A.seed_slots(4, 1)
    for k in range(4):
        ctx = A.Context(0)
        imgs = [A.synthetic_image(900 + 8 * k + i, 300, 280, 3) for i in range(8)]
        ps = [f.make_params(eng, 300, 280, 224, 224) for _ in imgs]
        info = {}
        got = H.hip_records(ctx, imgs, ps, od, info=info)
        ctx.close()
        for i, (g, r) in enumerate(zip(got, H.oracle_records(imgs, ps, od))):
            assert np.array_equal(g, r), (k, H.lost_lines_report(info["dst_ptr"], od.item_stride, i, g, r))
    cfg = dict(batch_size=4, random_seed=9, batch_major=False, etl=[C.IMAGE_224], augmentation=[C.C3_AUG])
    recs = _records(8, seed=4)
    for _ in range(2):
        (out,) = A.Decoder(cfg).decode(recs)
        (pin,) = _decode_pinned(A.Decoder(cfg), recs)
        assert np.array_equal(out.view(np.uint8), pin.view(np.uint8)), (
            _diff_report(out, pin), "uncached blocks: " + str([(hex(lo), hex(hi)) for lo, hi in A.uncached_blocks()]))
