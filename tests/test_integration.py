"""GPU: the aeon-side drop-in of INTEGRATION.md, emulated call for call through the C ABI.

aeon's batch_decoder::filler runs `process(index)` for index in [0, decode_size) on its pool
(src/batch_decoder.cpp:62-99); process calls

    m_provider->provide(index % batch_size, record(index), (*outputs)[index / batch_size])

where m_provider is a provider_base (src/provider_factory.cpp:24-51) whose provide() calls each ETL
provider with one shared `augmentation` (src/provider.cpp:109-119).  The one-line change adds, after
m_thread_pool.run, `for b: m_provider->post_process((*outputs)[b])`, and provider_base gains the
override that forwards post_process to each element of m_providers (src/provider.hpp:64-76).

The emulation below calls ONLY ProviderBase.provide (from 8 pool threads) and ProviderBase.post_process
(per batch, from the filler thread).  provider::image / provider::pixelmask hold an aeon_hip_stager:
provide() stages the decoded record under (its batch buffer, idx), post_process() flushes -- the first
flush of a window launches the whole window, one kernel launch over decode_size records.  Every batch
buffer of every window must equal the oracle bit for bit: C2, C3 (lighting: params drawn in record
order, aeon's one-thread order), and C5 (image + pixel mask sharing one params set), with pageable,
pinned (zero-copy) and device batch buffers.
"""
import ctypes
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu


class Buffer:
    """One buffer_fixed_size_elements of a batch (src/buffer_batch.hpp:154-188): pageable numpy,
    pinned host (aeon's "pinned" loader option) or device memory."""

    def __init__(self, nbytes, where):
        import torch
        self.where = where
        if where == "device":
            self.t = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
            self.ptr = self.t.data_ptr()
        elif where == "pinned":
            p = ctypes.c_void_p()
            A._check(A.lib().aeon_hip_host_alloc(nbytes, ctypes.byref(p)))
            self.ptr, self.n = p.value, nbytes
            ctypes.memset(self.ptr, 0, nbytes)
        else:
            self.a = np.zeros(nbytes, np.uint8)
            self.ptr = self.a.ctypes.data

    def bytes(self):
        if self.where == "device":
            return self.t.cpu().numpy()
        if self.where == "pinned":
            return np.ctypeslib.as_array((ctypes.c_uint8 * self.n).from_address(self.ptr)).copy()
        return self.a

    def free(self):
        if self.where == "pinned":
            A.lib().aeon_hip_host_free(ctypes.c_void_p(self.ptr))


class FixedBufferMap:
    """fixed_buffer_map of one batch: buffer name -> Buffer."""

    def __init__(self, shapes, batch, where):
        self.buf = {name: Buffer(batch * item, where) for name, item in shapes}

    def __getitem__(self, name):
        return self.buf[name]


class Augmentation:  # nervana::augmentation (src/provider.hpp:86-91)
    def __init__(self):
        self.image_params = None


class DrawOrder:
    """make_params in record order: lighting's normal_distribution caches a draw inside the shared
    factory, so aeon's result is defined by its one-thread order."""

    def __init__(self):
        self.cv = threading.Condition()
        self.next = 0

    def run(self, index, fn):
        with self.cv:
            self.cv.wait_for(lambda: self.next == index)
            try:
                return fn()
            finally:
                self.next += 1
                self.cv.notify_all()


class HipImageProvider:
    """provider::image, HIP flavour."""

    def __init__(self, ctx, etl, aug, batch, where, factory):
        self.name = "image"
        self.item = C.out_desc_for(etl, aug).item_stride
        self.w, self.h = etl["width"], etl["height"]
        self.factory = factory
        kind = A.STAGER_IMAGE | (A.STAGER_DEVICE_OUT if where == "device" else 0)
        self.stager = A.Stager(ctx, C.out_desc_for(etl, aug), batch, kind)

    def provide(self, idx, datum, out_buf, aug, engine, order, index):
        img = datum  # image::extractor::extract: the decoded record (unchanged, host)
        if aug.image_params is None:  # make_params (unchanged, host)
            aug.image_params = order.run(index, lambda: self.factory.make_params(engine, img.shape[1], img.shape[0],
                                                                                self.w, self.h))
        self.stager.stage(out_buf[self.name].ptr, idx, img, aug.image_params)

    def post_process(self, out_buf):
        self.stager.flush(out_buf[self.name].ptr)


class HipPixelmaskProvider(HipImageProvider):
    """provider::pixelmask, HIP flavour: the record's image params (src/provider.cpp:378-391)."""

    def __init__(self, ctx, etl, aug, batch, where, factory):
        self.name = "pixelmask"
        self.item = C.out_desc_for(etl, aug).item_stride
        self.w, self.h = etl["width"], etl["height"]
        self.factory = factory
        kind = A.STAGER_MASK | (A.STAGER_DEVICE_OUT if where == "device" else 0)
        self.stager = A.Stager(ctx, C.out_desc_for(etl, aug), batch, kind)


class ProviderBase:
    """provider_base with the forwarding post_process override."""

    def __init__(self, providers):
        self.providers = providers

    def provide(self, idx, record, out_buf, engine, order, index):
        aug = Augmentation()
        for k, p in enumerate(self.providers):
            p.provide(idx, record[k], out_buf, aug, engine, order, index)

    def post_process(self, out_buf):
        for p in self.providers:
            p.post_process(out_buf)


def _records(cfg, n, seed):
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(n):
        w, h = int(rng.integers(200, 640)), int(rng.integers(200, 640))
        img = A.synthetic_image(i + 10007 * seed, w, h, 3)
        if cfg == "C5":
            recs.append((img, rng.integers(0, 21, (h, w), dtype=np.uint8)))
        else:
            recs.append((img,))
    return recs


@pytest.mark.parametrize("cfg,where", [("C2", "pageable"), ("C3", "pageable"), ("C5", "pageable"),
                                       ("C2", "pinned"), ("C5", "pinned"), ("C3", "device")])
def test_provider_base_post_process_drop_in(cfg, where):
    aug = {"C2": C.C2_AUG, "C3": C.C3_AUG, "C5": C.C5_AUG}[cfg]
    etl = [C.IMAGE_512, C.MASK_512] if cfg == "C5" else [C.IMAGE_224]
    batch, nbatches, seed = (16, 4, 9) if cfg == "C5" else (32, 4, 7)
    decode_size = batch * nbatches
    ctx = A.Context(0)
    factory = A.ParamFactory(aug)
    kinds = [HipImageProvider, HipPixelmaskProvider]
    provs = [kinds[k](ctx, e, aug, batch, where, factory) for k, e in enumerate(etl)]
    base = ProviderBase(provs)
    shapes = [(p.name, p.item) for p in provs]
    engines = A.seed_slots(seed, decode_size)  # m_random (batch_decoder.cpp:47-54), kept across windows
    checker_states = engines.copy()
    bufs = []
    try:
        for window in range(2):  # the second window reuses every stager (pinned chunks, events)
            records = _records(cfg, decode_size, seed=window)
            outputs = [FixedBufferMap(shapes, batch, where) for _ in range(nbatches)]
            bufs += outputs
            order = DrawOrder()

            def process(index):  # batch_decoder::process
                eng = engines[index:index + 1]
                base.provide(index % batch, records[index], outputs[index // batch], eng, order, index)

            with ThreadPoolExecutor(max_workers=8) as pool:  # m_thread_pool.run(this, m_decode_size)
                list(pool.map(process, range(decode_size)))
            for b in range(nbatches):  # the one-line change in batch_decoder::filler
                base.post_process(outputs[b])

            # checker: the same draws in record order, the oracle per batch
            chk = A.ParamFactory(aug)
            params = []
            for i, r in enumerate(records):
                st = checker_states[i:i + 1]
                params.append(chk.make_params(st, r[0].shape[1], r[0].shape[0], etl[0]["width"], etl[0]["height"]))
            for k, (p, e) in enumerate(zip(provs, etl)):
                od = C.out_desc_for(e, aug)
                ref = H.oracle_records([r[k] for r in records], params, od, mask=(k == 1))
                dt = A.NP_DTYPE[od.dtype]
                for b in range(nbatches):
                    got = outputs[b][p.name].bytes().view(dt)
                    for i in range(batch):
                        item = got[i * (p.item // np.dtype(dt).itemsize):(i + 1) * (p.item // np.dtype(dt).itemsize)]
                        assert np.array_equal(item, ref[b * batch + i].reshape(-1)), (cfg, where, window, p.name, b, i)
    finally:
        for p in provs:
            p.stager.close()
        for o in bufs:
            for bf in o.buf.values():
                bf.free()
        ctx.close()


def test_stager_errors():
    """Flush without stages, an unknown batch buffer, a batch with a hole, a double stage."""
    ctx = A.Context(0)
    out = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
    st = A.Stager(ctx, out, 4)
    p = A.ParamFactory(C.C2_AUG).make_params(A.seed_slots(1, 1), 300, 300, 224, 224)
    buf = np.zeros(4 * out.item_stride, np.uint8)
    other = np.zeros(4 * out.item_stride, np.uint8)
    img = A.synthetic_image(0, 300, 300, 3)
    try:
        with pytest.raises(A.AeonHipError):
            st.flush(buf.ctypes.data)
        st.stage(buf.ctypes.data, 0, img, p)
        with pytest.raises(A.AeonHipError):
            st.stage(buf.ctypes.data, 0, img, p)  # idx staged twice
        st.stage(buf.ctypes.data, 2, img, p)  # idx 1 missing
        with pytest.raises(A.AeonHipError):
            st.flush(buf.ctypes.data)
        # the failed window was dropped whole: a fresh one works
        for i in range(4):
            st.stage(buf.ctypes.data, i, img, p)
        with pytest.raises(A.AeonHipError):
            st.flush(other.ctypes.data)  # not staged in this window (the window is launched by it)
        st.flush(buf.ctypes.data)
        ref = H.oracle_records([img], [p], out)[0]
        assert np.array_equal(buf[:out.item_stride].view(np.float32), ref.reshape(-1))
    finally:
        st.close()
        ctx.close()
