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
    pinned host (aeon's "pinned" loader option: buffer_fixed_size_elements::allocate's HAS_GPU branch,
    src/buffer_batch.cpp:150-186, as INTEGRATION.md edit 5 rewrites it -- aeon_hip_host_alloc /
    aeon_hip_host_free) or device memory."""

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

    overlap = False

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
        if self.overlap:  # launch only: the consumer waits (batch_iterator_fbm::filler edit)
            self.stager.launch(out_buf[self.name].ptr)
        else:
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
            st.flush(other.ctypes.data)  # not staged in this window
        st.flush(buf.ctypes.data)
        ref = H.oracle_records([img], [p], out)[0]
        assert np.array_equal(buf[:out.item_stride].view(np.float32), ref.reshape(-1))
    finally:
        st.close()
        ctx.close()


def _check_window(cfg, aug, etl, provs, records, checker_states, batch, nbatches, read):
    """Every batch of a window against the oracle; read(b, name) -> the batch buffer's bytes."""
    chk = A.ParamFactory(aug)
    params = []
    for i, r in enumerate(records):
        st = checker_states[i:i + 1]
        params.append(chk.make_params(st, r[0].shape[1], r[0].shape[0], etl[0]["width"], etl[0]["height"]))
        checker_states[i] = st[0]
    for k, (p, e) in enumerate(zip(provs, etl)):
        od = C.out_desc_for(e, aug)
        ref = H.oracle_records([r[k] for r in records], params, od, mask=(k == 1))
        dt = A.NP_DTYPE[od.dtype]
        n = p.item // np.dtype(dt).itemsize
        for b in range(nbatches):
            got = read(b, p.name).view(dt)
            for i in range(batch):
                assert np.array_equal(got[i * n:(i + 1) * n], ref[b * batch + i].reshape(-1)), (cfg, p.name, b, i)


@pytest.mark.parametrize("cfg,where", [("C2", "pageable"), ("C5", "pageable"), ("C3", "pinned"), ("C2", "device")])
def test_overlapped_windows_consumer_waits(cfg, where):
    """aeon's async_manager with the second aeon-side edit: the decode stage (batch_decoder::filler) runs
    provide() on its pool and post_process() per batch, which only LAUNCHES the window, and hands the
    container on; the consumer (batch_iterator_fbm::filler) calls aeon_hip_stager_wait(NULL, buffer) for
    every buffer of a batch before it copies the batch out.  Two containers alternate
    (src/async_manager.hpp:162-204), so window k's GPU work overlaps window k+1's provide() calls.  Four
    windows; every batch bit-exact against the oracle."""
    import queue
    aug = {"C2": C.C2_AUG, "C3": C.C3_AUG, "C5": C.C5_AUG}[cfg]
    etl = [C.IMAGE_512, C.MASK_512] if cfg == "C5" else [C.IMAGE_224]
    batch, nbatches, seed = (16, 4, 5) if cfg == "C5" else (32, 4, 3)
    decode_size, nwin = batch * nbatches, 4
    ctx = A.Context(0)
    factory = A.ParamFactory(aug)
    kinds = [HipImageProvider, HipPixelmaskProvider]
    provs = [kinds[k](ctx, e, aug, batch, where, factory) for k, e in enumerate(etl)]
    for p in provs:
        p.overlap = True
    base = ProviderBase(provs)
    shapes = [(p.name, p.item) for p in provs]
    containers = [[FixedBufferMap(shapes, batch, where) for _ in range(nbatches)] for _ in range(2)]
    engines = A.seed_slots(seed, decode_size)
    checker_states = engines.copy()
    free_q, full_q = queue.Queue(), queue.Queue()
    for c in range(2):
        free_q.put(c)
    all_records = [_records(cfg, decode_size, seed=100 + w) for w in range(nwin)]
    errors = []

    def decode_stage():  # async_manager::run_filler over batch_decoder::filler
        try:
            with ThreadPoolExecutor(max_workers=8) as pool:
                for w in range(nwin):
                    c = free_q.get()
                    outputs, records, order = containers[c], all_records[w], DrawOrder()

                    def process(index):
                        eng = engines[index:index + 1]
                        base.provide(index % batch, records[index], outputs[index // batch], eng, order, index)

                    list(pool.map(process, range(decode_size)))
                    for b in range(nbatches):
                        base.post_process(outputs[b])  # launch only
                    full_q.put((w, c))
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append(e)
            full_q.put(None)

    th = threading.Thread(target=decode_stage)
    th.start()
    try:
        for _ in range(nwin):  # batch_iterator_fbm::filler, per decoded container
            item = full_q.get(timeout=120)
            assert item is not None, errors
            w, c = item
            copies = {}
            for b in range(nbatches):
                for name, _ in shapes:
                    buf = containers[c][b][name]
                    A.Stager.wait_buffer(buf.ptr)  # the second aeon-side edit
                    copies[(b, name)] = buf.bytes().copy()  # the swap / copy out of the container
            free_q.put(c)  # the container goes back to the decode stage
            _check_window(cfg, aug, etl, provs, all_records[w], checker_states, batch, nbatches,
                          lambda b, name: copies[(b, name)])
        th.join(timeout=120)
        assert not errors, errors
    finally:
        th.join(timeout=120)
        for p in provs:
            p.stager.close()
        for cont in containers:
            for o in cont:
                for bf in o.buf.values():
                    bf.free()
        ctx.close()


def test_stager_launch_wait_errors():
    """launch() of a batch staged in no window; a second launch of one batch; wait() of a buffer no stager
    launched returns at once; a third window staged while the first was never waited for drops the first."""
    ctx = A.Context(0)
    out = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
    st = A.Stager(ctx, out, 2)
    f = A.ParamFactory(C.C2_AUG)
    p = f.make_params(A.seed_slots(1, 1), 300, 300, 224, 224)
    img = A.synthetic_image(3, 300, 300, 3)
    bufs = [np.zeros(2 * out.item_stride, np.uint8) for _ in range(3)]
    ref = H.oracle_records([img], [p], out)[0].reshape(-1)
    try:
        with pytest.raises(A.AeonHipError):
            st.launch(bufs[0].ctypes.data)
        A.Stager.wait_buffer(bufs[0].ctypes.data)  # nothing launched it: returns
        for w in range(3):  # windows 0, 1, 2 on one buffer each; nobody waits for 0 and 1
            for i in range(2):
                st.stage(bufs[w].ctypes.data, i, img, p)
            st.launch(bufs[w].ctypes.data)
            with pytest.raises(A.AeonHipError):
                st.launch(bufs[w].ctypes.data)  # twice in one window
        st.wait(bufs[2].ctypes.data)
        for w in range(3):  # window 0 was completed when window 2 staged; 1 and 2 by their waits
            A.Stager.wait_buffer(bufs[w].ctypes.data)
            for i in range(2):
                assert np.array_equal(bufs[w][i * out.item_stride:(i + 1) * out.item_stride].view(np.float32), ref), (w, i)
    finally:
        st.close()
        ctx.close()


def test_aeon_path_cpp_native_sequence():
    """tools/aeon_path_cpp.cpp (INTEGRATION.md edits 1-5 in C++ against the C ABI alone): a short run of
    each form -- pinned (edit 5: zero-copy stores) and pageable batch buffers, launch-only post_process with
    the consumer's waits, and flushing post_process -- completes and reports its rate.  (Its outputs are the
    stager's, which the tests above check bit for bit through the same entry points.)"""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "aeon_amd", "aeon_path_cpp")
    assert os.path.exists(exe), "aeon_amd/aeon_path_cpp not built (make -C aeon_amd/csrc)"
    for buffers in ("pinned", "pageable"):
        for mode in ("overlap", "flush"):
            r = subprocess.run([exe, "C2", buffers, mode, "2", "1"], capture_output=True, text=True, timeout=120)
            assert r.returncode == 0, r.stderr
            line = json.loads(r.stdout.strip().splitlines()[-1])
            assert line["buffers"] == buffers and line["value"] > 0, line
