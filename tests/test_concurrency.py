"""GPU: one context driven from several host threads at once (the verdict's concurrent-caller case).

aeon's loader holds one provider::image and one provider::pixelmask per decode stage, and a host may
run more than one stage per process: their calls reach one aeon_hip_ctx from different threads.  The
context serialises a call's host half under its mutex (ring slot, job table written into HBM through
the BAR by that one thread, read back before the launch -- stage.cpp publish_table), then the kernels
run on the caller's stream.  Here three threads hammer one context together:

  * an image stager (C2 params, pageable batch buffers: one launch per window + D2H per batch),
  * a pixel-mask stager (C5 masks, pinned batch buffers: zero-copy stores),
  * direct aeon_hip_augment_batch calls on a torch stream of their own (C2, device outputs),

each for several windows / calls, and every output is checked against the oracle afterwards.
"""
import ctypes
import threading

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu


class Pinned:
    """A pinned, device-mapped host batch buffer (aeon_hip_host_alloc: the kernels store into it)."""

    def __init__(self, nbytes):
        p = ctypes.c_void_p()
        A._check(A.lib().aeon_hip_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr, self.n = p.value, nbytes
        ctypes.memset(self.ptr, 0, nbytes)

    def bytes(self):
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.n).from_address(self.ptr))

    def free(self):
        A.lib().aeon_hip_host_free(ctypes.c_void_p(self.ptr))


def test_three_threads_one_context():
    import torch
    ctx = A.Context(0)
    errors, results = [], {}
    img_out = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
    mask_out = C.out_desc_for(C.MASK_512, C.C5_AUG)

    def image_stager():
        st = A.Stager(ctx, img_out, 8)
        f = A.ParamFactory(C.C2_AUG)
        eng = A.seed_slots(3, 1)
        try:
            for w in range(6):
                imgs = [A.synthetic_image(100 * w + i, 300 + 7 * i, 280 + 5 * i, 3) for i in range(16)]
                ps = [f.make_params(eng, m.shape[1], m.shape[0], 224, 224) for m in imgs]
                bufs = [np.zeros(8 * img_out.item_stride, np.uint8) for _ in range(2)]
                for i, (m, p) in enumerate(zip(imgs, ps)):
                    st.stage(bufs[i // 8].ctypes.data, i % 8, m, p)
                for b in bufs:
                    st.flush(b.ctypes.data)
                results[("image", w)] = (imgs, ps, [b.copy() for b in bufs])
        except Exception as e:  # noqa: BLE001
            errors.append(e)
        finally:
            st.close()

    def mask_stager():
        st = A.Stager(ctx, mask_out, 4, A.STAGER_MASK)
        f = A.ParamFactory(C.C5_AUG)
        eng = A.seed_slots(5, 1)
        bufs = []
        try:
            for w in range(6):
                masks = [np.random.default_rng(w * 10 + i).integers(0, 21, (400 + 9 * i, 420 + 3 * i), dtype=np.uint8)
                         for i in range(8)]
                ps = [f.make_params(eng, m.shape[1], m.shape[0], 512, 512) for m in masks]
                wb = [Pinned(4 * mask_out.item_stride) for _ in range(2)]
                bufs += wb
                for i, (m, p) in enumerate(zip(masks, ps)):
                    st.stage(wb[i // 4].ptr, i % 4, m, p)
                for b in wb:
                    st.flush(b.ptr)
                results[("mask", w)] = (masks, ps, [b.bytes().copy() for b in wb])
        except Exception as e:  # noqa: BLE001
            errors.append(e)
        finally:
            st.close()
            for b in bufs:
                b.free()

    def direct_calls():
        try:
            s = torch.cuda.Stream()
            f = A.ParamFactory(C.C2_AUG)
            eng = A.seed_slots(9, 1)
            for k in range(8):
                imgs = [A.synthetic_image(5000 + 40 * k + i, 256, 256, 3) for i in range(24)]
                ps = [f.make_params(eng, 256, 256, 224, 224) for _ in imgs]
                with torch.cuda.stream(s):  # (hip_records launches on the current stream)
                    res = H.hip_records(ctx, imgs, ps, img_out)
                results[("direct", k)] = (imgs, ps, res)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def check():
        bad = []
        for (kind, w), (srcs, ps, got) in sorted(results.items()):
            if kind == "direct":
                ref = H.oracle_records(srcs, ps, img_out)
                for i, (g, r) in enumerate(zip(got, ref)):
                    if not np.array_equal(g, r):
                        bad.append((kind, w, i, int((g != r).sum()), int(g.size)))
                continue
            od = img_out if kind == "image" else mask_out
            ref = H.oracle_records(srcs, ps, od, mask=(kind == "mask"))
            per = len(srcs) // len(got)
            dt = A.NP_DTYPE[od.dtype]
            n = od.item_stride // np.dtype(dt).itemsize
            for i, r in enumerate(ref):
                item = got[i // per].view(dt)[(i % per) * n:(i % per + 1) * n]
                if not np.array_equal(item, r.reshape(-1)):
                    bad.append((kind, w, i, int((item != r.reshape(-1)).sum()), int(item.size),
                                int((item == 0).sum())))
        return bad

    try:
        # each worker alone first, then the three at once
        for t in (image_stager, mask_stager, direct_calls):
            t()
        assert not errors, errors
        bad_serial = check()
        results.clear()
        ths = [threading.Thread(target=t) for t in (image_stager, mask_stager, direct_calls)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=300)
        assert not errors, errors
        assert len(results) == 6 + 6 + 8
        bad = check()
        assert not bad_serial and not bad, (bad_serial[:8], bad[:8], len(bad_serial), len(bad))
    finally:
        ctx.close()
