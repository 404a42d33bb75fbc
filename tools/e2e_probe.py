"""Host->host C2 rate with the kernel reading / writing pinned host memory directly (zero-copy over
PCIe) against bench.run_e2e's H2D copy -> kernel -> D2H copy pipeline.  Development probe:
python tools/e2e_probe.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import aeon_amd as A  # noqa: E402
import bench  # noqa: E402
from aeon_amd import configs as C  # noqa: E402


def device_view(t):
    """The device address of a pinned host tensor (hipHostGetDevicePointer through torch's own HIP
    runtime); refuses to go on unless the buffer is device-mapped."""
    import ctypes
    hip = ctypes.CDLL(os.path.join(torch.__path__[0], "lib", "libamdhip64.so"))
    d = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(t.data_ptr()), 0)
    if rc != 0 or not d.value:
        raise RuntimeError("pinned buffer is not device-mapped (hipHostGetDevicePointer rc %d)" % rc)
    return d.value


def direct(batch, steps, src_on_host, nbuf=2):
    ctx = A.Context(torch.cuda.current_device())
    w = h = 256
    img_bytes = w * h * 3
    out = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
    host_src = [torch.randint(0, 256, (batch * img_bytes,), dtype=torch.uint8).pin_memory() for _ in range(nbuf)]
    host_dst = [torch.empty(batch * out.item_stride, dtype=torch.uint8).pin_memory() for _ in range(nbuf)]
    dev_src = [torch.empty(batch * img_bytes, dtype=torch.uint8, device="cuda") for _ in range(nbuf)]
    descs = (A.ImgDesc * batch)(*[A.ImgDesc(offset=i * img_bytes, width=w, height=h, stride=w * 3, channels=3)
                                  for i in range(batch)])
    f = A.ParamFactory(C.C2_AUG)
    states = A.seed_slots(1, batch)
    params = [(A.AugParams * batch)(*[f.make_params(states[i:i + 1], w, h, 224, 224) for i in range(batch)])
              for _ in range(4)]
    src_dev_view = [device_view(t) for t in host_src]
    dst_dev_view = [device_view(t) for t in host_dst]
    print("device views equal host addresses:", all(device_view(t) == t.data_ptr() for t in host_src + host_dst))
    s_h2d, s_k = torch.cuda.Stream(), torch.cuda.Stream()
    ev_in = [torch.cuda.Event() for _ in range(nbuf)]
    ev_k = [torch.cuda.Event() for _ in range(nbuf)]

    def one(s):
        j = s % nbuf
        if src_on_host:
            src = src_dev_view[j]
        else:
            with torch.cuda.stream(s_h2d):
                s_h2d.wait_event(ev_k[j])
                dev_src[j].copy_(host_src[j], non_blocking=True)
                ev_in[j].record(s_h2d)
            s_k.wait_event(ev_in[j])
            src = dev_src[j].data_ptr()
        ctx.augment_batch(descs, src, params[s % 4], out, dst_dev_view[j], s_k.cuda_stream)
        ev_k[j].record(s_k)

    for s in range(nbuf):
        one(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        one(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.close()
    return batch * steps / dt


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    torch.cuda.set_device(0)
    print("copies (bench.run_e2e)", round(bench.run_e2e(A, C, torch, 256, steps)), flush=True)
    print("kernel writes pinned host", round(direct(256, steps, False)), flush=True)
    print("kernel reads + writes pinned host", round(direct(256, steps, True)), flush=True)
