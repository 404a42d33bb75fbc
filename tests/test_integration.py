"""GPU: the aeon-side integration sketch of INTEGRATION.md, emulated call for call through the C ABI.

aeon's batch_decoder::filler runs `process(index)` for index in [0, decode_size) on its pool
(src/batch_decoder.cpp:62-99), and process calls

    provide(index % batch_size, record(index), (*outputs)[index / batch_size])

so a provider sees only `idx` (repeating once per batch of the window) and the batch's own
fixed_buffer_map.  The HIP provider below mirrors the INTEGRATION.md C++ sketch: provide() stages
the decoded record + its params under the key (that batch's buffer map, idx); the post_process hook,
called once per batch after the pool finishes, uploads that batch's staging, runs
aeon_hip_augment_batch into a device buffer and copies it into that batch's buffer.  Every batch
buffer of a decode_size = 4 x batch window must equal the oracle bit for bit.
"""
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import aeon_amd as A
from aeon_amd import configs as C
from tests import helpers as H

pytestmark = pytest.mark.gpu


class FixedBufferMap:
    """One batch of a window's array_fixed_buffer_map: the 'image' buffer, batch items."""

    def __init__(self, batch, item_shape):
        self.image = np.zeros((batch,) + item_shape, np.float32)


class HipImageProvider:
    """provider::image, HIP flavour: staging keyed by (batch buffer, idx)."""

    def __init__(self, ctx, aug, etl, batch):
        self.ctx, self.batch = ctx, batch
        self.factory = A.ParamFactory(aug)
        self.lock = threading.Lock()  # guards the key map
        # make_params' lighting draws share the factory's normal_distribution, whose cached second
        # value makes a record's draw depend on the previous one (aeon's threaded draws race on it,
        # SURVEY.md §8(b)); the draws are taken in record order, as aeon_decoder does and as aeon
        # does on one thread
        self.turn = threading.Condition()
        self.next_draw = 0
        self.out = C.out_desc_for(etl, aug)
        self.w, self.h = etl["width"], etl["height"]
        self.stage = {}  # id(batch buffer map) -> [(image, params)] * batch

    def _batch_stage(self, out_buf):
        with self.lock:
            return self.stage.setdefault(id(out_buf), [None] * self.batch)

    def provide(self, idx, record, out_buf, engine, index):
        img = record  # extract: already decoded (unchanged, host)
        with self.turn:  # make_params (unchanged, host) on the record's slot engine, in record order
            self.turn.wait_for(lambda: self.next_draw == index)
            p = self.factory.make_params(engine, img.shape[1], img.shape[0], self.w, self.h)
            self.next_draw += 1
            self.turn.notify_all()
        self._batch_stage(out_buf)[idx] = (img, p)

    def post_process(self, out_buf):
        import torch
        staged = self.stage.pop(id(out_buf))
        arena, descs = A.pack_images([s[0] for s in staged])
        dev_src = torch.from_numpy(arena).to("cuda", non_blocking=False)  # H2D of this batch's staging
        dev_out = torch.empty(self.batch * self.out.item_stride, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        self.ctx.augment_batch(descs, dev_src.data_ptr(), [s[1] for s in staged], self.out, dev_out.data_ptr(),
                               stream)
        host = dev_out.cpu().numpy()  # D2H into this batch's buffer
        out_buf.image[...] = host.view(np.float32).reshape(out_buf.image.shape)
        self.ctx.synchronize(stream)


@pytest.mark.parametrize("aug_name", ["C2", "C3"])
def test_integration_sketch_call_pattern(aug_name):
    aug = {"C2": C.C2_AUG, "C3": C.C3_AUG}[aug_name]
    batch, nbatches, seed = 32, 4, 7
    decode_size = batch * nbatches
    rng = np.random.default_rng(5)
    records = [A.synthetic_image(i, int(rng.integers(200, 600)), int(rng.integers(200, 600)), 3)
               for i in range(decode_size)]
    ctx = A.Context(0)
    try:
        prov = HipImageProvider(ctx, aug, C.IMAGE_224, batch)
        outputs = [FixedBufferMap(batch, (3, 224, 224)) for _ in range(nbatches)]
        engines = A.seed_slots(seed, decode_size)  # m_random (batch_decoder.cpp:47-54)

        def process(index):  # batch_decoder::process
            eng = engines[index:index + 1]
            prov.provide(index % batch, records[index], outputs[index // batch], eng, index)

        with ThreadPoolExecutor(max_workers=8) as pool:  # m_thread_pool.run(this, m_decode_size)
            list(pool.map(process, range(decode_size)))
        for b in range(nbatches):  # the one-line change: post_process per batch of the window
            prov.post_process(outputs[b])
    finally:
        ctx.close()
    params = H.draw_params(aug, [(r.shape[1], r.shape[0]) for r in records], 224, 224, seed=seed)
    out = C.out_desc_for(C.IMAGE_224, aug)
    for b in range(nbatches):
        ref = H.oracle_records(records[b * batch:(b + 1) * batch], params[b * batch:(b + 1) * batch], out)
        for i in range(batch):
            assert np.array_equal(outputs[b].image[i], ref[i]), (aug_name, b, i)
