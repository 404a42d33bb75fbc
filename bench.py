#!/usr/bin/env python3
"""Benchmark of the MI355X image-augmentation stage (BASELINE.json metric).

A "step" = one decode window of `batch` records through the HIP stage: random crop + flip +
bilinear resize to 224x224 (+ photometric for C3), standardize, CHW fp32, with the decoded
HWC uint8 sources already resident in HBM (device-resident metric).  The source pool spans
more than the 256 MiB Infinity Cache so every step streams its sources from HBM.
Augmentation parameters come from aeon's deterministic mode (random_seed 1 + node_id,
one minstd_rand0 per decode slot) and are drawn on the host before the timed region.

N GPUs: one process per GPU (torch.distributed.run), each an independent manifest slice
(node_id = rank, node_count = N, aeon src/manifest_file.cpp:278-295) with decoder seed
random_seed + node_id (src/loader.cpp:174): no data-path collective; barrier + max-over-ranks
timing.  `python bench.py --gpus N` with no torchrun environment starts torchrun itself as a
child process (this parent never touches the GPU).  At N > 1 the line also carries C4 (the C3
workload at per-GPU batch 1024 on every rank).  --dry-run rehearses the launcher, the slicing
and the seeding with gloo on the CPU (no GPU work).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "augmented images/s device-resident, 224×224 batch 256; achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C2", choices=["C2", "C3"])
    ap.add_argument("--batch", type=int, default=0, help="records per step (default: config's)")
    ap.add_argument("--pool-mib", type=int, default=400, help="source pool size per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3 and end-to-end side runs")
    ap.add_argument("--streams", type=int, default=1, help="development: alternate batches over N streams")
    ap.add_argument("--timing-every", type=int, default=0,
                    help="development: also bracket the kernels of one step in N with HIP events (0 = none; the "
                         "roofline's duration comes from one event pair around the timed region's launches, "
                         "run_device(region=True)); each timed launch idles the queue ~9 us around it")
    ap.add_argument("--cpu-extra-seconds", type=float, default=3.0,
                    help="CPU-baseline sample budget of each of C1/C3/C5")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_r05p.json"))
    ap.add_argument("--share-device", action="store_true",
                    help="development: ranks share the visible GPUs round-robin (gloo barrier), to run "
                         "the N-rank path on a 1-GPU box")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the N-rank path (gloo, no GPU): slices, seeds, timing")
    return ap.parse_args()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """--gpus N without a torchrun environment: run torchrun with N ranks as a CHILD process
    (never exec: this parent has not initialised the GPU and does not) and exit with its code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.call(cmd, env=env)


def rank_slice(n_records, batch, rank, world):
    """The record indices of this rank's manifest slice (aeon node slicing) and its decoder
    seed (random_seed 1 + node_id)."""
    import aeon_amd as A
    return A.manifest_node_slice(n_records, batch, rank, world), 1 + rank


def cpu_list_str(cpus):
    """[0, 1, 2, 5] -> "0-2,5" (aeon's cpu_list syntax, src/util.cpp:283-330)."""
    out, cpus = [], sorted(set(cpus))
    i = 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def parse_cpulist(text):
    cpus = set()
    for tok in text.strip().split(","):
        if not tok:
            continue
        a, _, b = tok.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def gpu_local_cpus(torch, device):
    """The CPUs of GPU `device`'s NUMA node (sysfs local_cpulist of its PCI function), or None."""
    try:
        p = torch.cuda.get_device_properties(device)
        addr = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{addr}/local_cpulist") as f:
            cpus = parse_cpulist(f.read())
        return cpus or None
    except (OSError, ValueError, AttributeError, RuntimeError):
        return None


def rank_cpu_lists(local, allowed, world):
    """Disjoint per-rank decode-pool cpu lists for one process per GPU (aeon pins each pool worker to
    one CPU of its cpu_list, src/thread_pool.hpp:133-138): rank r prefers the CPUs of its GPU's NUMA
    node that this process may use (local[r]; None = unknown -> any allowed CPU).  The allowed CPUs are
    shared out as evenly as the preferences permit (one CPU per rank in turn), then each rank takes its
    count of the lowest free CPUs of its preference, so ranks of one node get contiguous blocks.  With
    more ranks than CPUs a rank without one shares a CPU of its preference."""
    allowed = sorted(allowed)
    pref = []
    for r in range(world):
        loc = local[r] if r < len(local) else None
        p = sorted(set(loc) & set(allowed)) if loc else []
        pref.append(p or allowed)
    free, counts = set(allowed), [0] * world
    progress = True
    while free and progress:
        progress = False
        for r in range(world):
            c = next((x for x in pref[r] if x in free), None)
            if c is None:
                c = min(free) if free else None
            if c is not None:
                free.discard(c)
                counts[r] += 1
                progress = True
    free, out = set(allowed), []
    for r in range(world):
        mine = [x for x in pref[r] if x in free][:counts[r]]
        if len(mine) < counts[r]:
            mine += sorted(free - set(mine))[:counts[r] - len(mine)]
        free -= set(mine)
        out.append(sorted(mine) or [pref[r][r % len(pref[r])]])
    return out


def synthetic_pool(torch, records, w, h, cn=3, seed=0x5EED, chunk=64, device="cuda"):
    """A.synthetic_image(g, w, h, cn) for every global record index g, computed on the device:
    splitmix64 in int64 arithmetic (wrapping add/mul; logical shifts by masking)."""
    n = len(records)
    L = w * h * cn
    out = torch.empty(n * L, dtype=torch.uint8, device=device)
    idx = torch.arange(L, dtype=torch.int64, device=device)

    def shr(z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)

    def s64(v):  # uint64 constant as the int64 with the same bits
        return v - (1 << 64) if v >= 1 << 63 else v

    g = torch.as_tensor(records, dtype=torch.int64, device=device)
    for a in range(0, n, chunk):
        gg = g[a:a + chunk, None]
        z = (seed ^ (gg << 32) ^ idx[None, :]) + s64(0x9E3779B97F4A7C15)
        z = (z ^ shr(z, 30)) * s64(0xBF58476D1CE4E5B9)
        z = (z ^ shr(z, 27)) * s64(0x94D049BB133111EB)
        z = z ^ shr(z, 31)
        out[a * L:(a + gg.shape[0]) * L] = (z & 0xFF).to(torch.uint8).reshape(-1)
    return out


def real_pool(torch, n, w, h):
    """n HWC u8 w x h sources cut from aeon's decoded img_2112_70.jpg (tests/golden, 480x360 BGR) at
    offsets that vary per record (natural-image statistics for the hue tables' LDS access pattern)."""
    img = np.load(os.path.join(ROOT, "tests", "golden", "img_2112_70_bgr.npz"))["bgr"]
    big = np.tile(img, (2, 2, 1))  # 960 x 720
    H, W = big.shape[:2]
    rng = np.random.default_rng(70)
    wins = [big[y:y + h, x:x + w] for x, y in zip(rng.integers(0, W - w, 64), rng.integers(0, H - h, 64))]
    base = torch.from_numpy(np.stack(wins).reshape(-1).copy()).to("cuda")
    reps = (n + 63) // 64
    return base.repeat(reps)[:n * w * h * 3].contiguous()


class Workload:
    """Synthetic already-decoded sources in HBM + pre-drawn params for every step."""

    def __init__(self, A, C, torch, cfg, batch, steps, rank, pool_mib, src_wh=(256, 256), world=1, real=False):
        self.batch = batch
        # "C2:CUBIC" etc.: the C2 workload with image::config's interpolation_method (the generic
        # resize pre-pass, resize_kernels.hip)
        base, _, interp = cfg.partition(":")
        self.aug = dict({"C2": C.C2_AUG, "C3": C.C3_AUG}[base])
        if interp:
            self.aug["interpolation_method"] = interp
        w, h = src_wh
        img_bytes = w * h * 3
        per_batch = batch * img_bytes
        self.n_pool = max(1, (pool_mib << 20) // per_batch)
        # this rank's records: its aeon node slice of a manifest of n_pool*batch*world records;
        # pixels = A.synthetic_image(global record index) generated on the device
        records, seed = rank_slice(self.n_pool * batch * world, batch, rank, world)
        self.src = synthetic_pool(torch, records[:self.n_pool * batch], w, h)
        if real:  # natural-image pixels instead: windows of aeon's img_2112_70.jpg record, tiled
            self.src = real_pool(torch, self.n_pool * batch, w, h)
        self.descs = [(A.ImgDesc * batch)(*[A.ImgDesc(offset=(b * batch + i) * img_bytes, width=w, height=h,
                                                      stride=w * 3, channels=3) for i in range(batch)])
                      for b in range(self.n_pool)]
        self.out = C.out_desc_for(C.IMAGE_224, self.aug)
        self.dst = [torch.empty(batch * self.out.item_stride, dtype=torch.uint8, device="cuda")
                    for _ in range(2)]
        # aeon deterministic mode: decoder seed = random_seed + node_id (src/loader.cpp:174),
        # one engine per decode slot, persisting across windows (src/batch_decoder.cpp:47-70)
        f = A.ParamFactory(self.aug)
        states = A.seed_slots(seed, batch)
        t0 = time.perf_counter()
        self.params = []
        for s in range(steps):
            ps = []
            for i in range(batch):
                st = states[i:i + 1]
                ps.append(f.make_params(st, w, h, 224, 224))
                states[i] = st[0]
            self.params.append((A.AugParams * batch)(*ps))  # marshalled once, as aeon's host fills it
        self.param_us = (time.perf_counter() - t0) / max(1, steps * batch) * 1e6

    def step(self, ctx, s, stream):
        # (device addresses read once: aeon's host holds plain pointers, not torch tensors)
        if not hasattr(self, "_ptrs"):
            self._ptrs = (self.src.data_ptr(), [d.data_ptr() for d in self.dst])
        b = s % self.n_pool
        ctx.augment_batch(self.descs[b], self._ptrs[0], self.params[s], self.out, self._ptrs[1][s & 1], stream)


def step_bytes(params):
    """Algorithmic bytes of one single-pass step (stage.cpp launch_bytes): each record's
    crop read once (u8 HWC) + its float32 CHW output written once."""
    return float(sum(p.crop_w * p.crop_h * 3 + p.out_w * p.out_h * 3 * 4 for p in params))


def run_device(A, C, torch, cfg, batch, steps, warmup, rank, world, pool_mib, dist, timing=8, streams=1,
               region=False, real=False):
    """region: time the kernels as the timed region runs them, back to back -- one HIP event pair on
    the launch stream around steps 2..K (the first step only fills the queue), kt['augment'] = (that
    span, the steps' algorithmic bytes, K - 1).  A step of this workload is one tile-kernel launch
    (single-pass calls: no planner, upload or copy ahead of it), so the span / (K - 1) is the average
    launch duration with each launch following the previous one, as rocprofv3 sees them; per-launch
    event pairs (timing) idle the queue around the launch they bracket and time it on a GPU that
    has drained the previous launch's stores (~8 % shorter)."""
    ctx = A.Context(torch.cuda.current_device())
    wl = Workload(A, C, torch, cfg, batch, steps + warmup, rank, pool_mib, world=world, real=real)
    # streams > 1 (development): consecutive batches alternate between caller streams, as a
    # loader double-buffering its output batches would
    # the launches go to a stream of our own (non-blocking, as a loader's would be): HIP's legacy null
    # stream synchronises with every blocking stream, which costs each launch host time
    prev_stream = torch.cuda.current_stream()
    torch.cuda.set_stream(torch.cuda.Stream())
    strs = [torch.cuda.current_stream().cuda_stream] + [torch.cuda.Stream().cuda_stream for _ in range(streams - 1)]
    stream = strs[0]
    for s in range(warmup):
        wl.step(ctx, s, strs[s % streams])
    torch.cuda.synchronize()
    ctx.kernel_times()  # drop warmup timings
    ctx.set_timing(timing)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if region else None
    t0 = time.perf_counter()
    call_s = []
    for s in range(warmup, warmup + steps):
        tc = time.perf_counter()
        wl.step(ctx, s, strs[s % streams])
        call_s.append(time.perf_counter() - tc)
        if region and s == warmup:
            ev[0].record(torch.cuda.current_stream())  # (strs[0] is the current stream)
    if region:
        ev[1].record(torch.cuda.current_stream())
    # host time per call: the median call (once the host is a ring of 16 calls ahead of the GPU, a
    # call also waits for a slot: the mean then follows the GPU, not the host's own cost)
    wl.submit_s = sorted(call_s)[len(call_s) // 2] * steps
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    for st in strs:
        ctx.synchronize(st)
    kt = ctx.kernel_times()
    ctx.set_timing(False)
    if region and steps > 1 and streams == 1:
        kt["augment"] = (ev[0].elapsed_time(ev[1]),
                         sum(step_bytes(wl.params[s]) for s in range(warmup + 1, warmup + steps)), steps - 1)
    if dist:
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ctx.close()
    torch.cuda.set_stream(prev_stream)
    return elapsed, kt, wl.param_us, wl.submit_s


def run_e2e(A, C, torch, batch, steps, zero_copy=False):
    """Host->host rate: pinned decoded pixels -> H2D -> kernel -> D2H into a pinned batch
    buffer, with copies and kernels on separate streams (PCIe-inclusive).  zero_copy:
    the kernel stores straight into the pinned batch buffer over PCIe (no device output, no D2H)."""
    ctx = A.Context(torch.cuda.current_device())
    w = h = 256
    img_bytes = w * h * 3
    out = C.out_desc_for(C.IMAGE_224, C.C2_AUG)
    host_src = [torch.randint(0, 256, (batch * img_bytes,), dtype=torch.uint8).pin_memory() for _ in range(2)]
    host_dst = [torch.empty(batch * out.item_stride, dtype=torch.uint8).pin_memory() for _ in range(2)]
    dev_src = [torch.empty(batch * img_bytes, dtype=torch.uint8, device="cuda") for _ in range(2)]
    dev_dst = [torch.empty(batch * out.item_stride, dtype=torch.uint8, device="cuda") for _ in range(2)]
    descs = (A.ImgDesc * batch)(*[A.ImgDesc(offset=i * img_bytes, width=w, height=h, stride=w * 3, channels=3)
                                  for i in range(batch)])
    f = A.ParamFactory(C.C2_AUG)
    states = A.seed_slots(1, batch)
    params = [(A.AugParams * batch)(*[f.make_params(states[i:i + 1], w, h, 224, 224) for i in range(batch)])
              for _ in range(4)]
    s_h2d, s_k, s_d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    ev_in = [torch.cuda.Event() for _ in range(2)]
    ev_k = [torch.cuda.Event() for _ in range(2)]
    ev_out = [torch.cuda.Event() for _ in range(2)]

    def one(s):
        j = s & 1
        with torch.cuda.stream(s_h2d):
            s_h2d.wait_event(ev_k[j])  # previous kernel on this buffer done reading
            dev_src[j].copy_(host_src[j], non_blocking=True)
            ev_in[j].record(s_h2d)
        s_k.wait_event(ev_in[j])
        s_k.wait_event(ev_out[j])  # previous D2H of this buffer done
        dst = host_dst[j].data_ptr() if zero_copy else dev_dst[j].data_ptr()
        ctx.augment_batch(descs, dev_src[j].data_ptr(), params[s % 4], out, dst, s_k.cuda_stream)
        ev_k[j].record(s_k)
        if zero_copy:
            return
        with torch.cuda.stream(s_d2h):
            s_d2h.wait_event(ev_k[j])
            host_dst[j].copy_(dev_dst[j], non_blocking=True)
            ev_out[j].record(s_d2h)

    for s in range(2):
        one(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        one(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.close()
    return batch * steps / dt


def run_c5(A, C, torch, steps, warmup, pool_mib, src_wh=(640, 480), kernel_timing=True):
    """C5 (BASELINE configs[4]): image + pixel mask drawn with ONE shared params set per record
    (aeon provider_base::provide, src/provider.cpp:109-119): joint crop/flip, bilinear image
    -> 512x512x3 f32 CHW, NEAREST mask -> 512x512x1 u8, batch 128, device-resident sources."""
    ctx = A.Context(torch.cuda.current_device())
    batch = C.CONFIGS["C5"]["batch_size"]
    w, h = src_wh
    ib, mb = w * h * 3, w * h
    n_pool = max(1, (pool_mib << 20) // (batch * (ib + mb)))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0x5EED5)
    img = torch.randint(0, 256, (n_pool * batch * ib,), dtype=torch.uint8, device="cuda", generator=gen)
    msk = torch.randint(0, 21, (n_pool * batch * mb,), dtype=torch.uint8, device="cuda", generator=gen)
    idescs = [(A.ImgDesc * batch)(*[A.ImgDesc(offset=(b * batch + i) * ib, width=w, height=h, stride=w * 3,
                                              channels=3) for i in range(batch)]) for b in range(n_pool)]
    mdescs = [(A.ImgDesc * batch)(*[A.ImgDesc(offset=(b * batch + i) * mb, width=w, height=h, stride=w,
                                              channels=1) for i in range(batch)]) for b in range(n_pool)]
    iout = C.out_desc_for(C.IMAGE_512, C.C5_AUG)
    mout = C.out_desc_for(C.MASK_512, C.C5_AUG)
    idst = [torch.empty(batch * iout.item_stride, dtype=torch.uint8, device="cuda") for _ in range(2)]
    mdst = [torch.empty(batch * mout.item_stride, dtype=torch.uint8, device="cuda") for _ in range(2)]
    f = A.ParamFactory(C.C5_AUG)
    states = A.seed_slots(1, batch)
    params = []
    for _ in range(steps + warmup):
        ps = []
        for i in range(batch):
            st = states[i:i + 1]
            ps.append(f.make_params(st, w, h, 512, 512))
            states[i] = st[0]
        params.append((A.AugParams * batch)(*ps))
    stream = torch.cuda.Stream().cuda_stream  # (a stream of our own: see run_device)

    separate = os.environ.get("AEON_BENCH_C5_SEPARATE") == "1"  # (A/B: the two calls of round 4)

    def step(s):  # provider::image + provider::pixelmask of the batch: one pair call
        b = s % n_pool
        if separate:
            ctx.augment_batch(idescs[b], img.data_ptr(), params[s], iout, idst[s & 1].data_ptr(), stream)
            ctx.mask_batch(mdescs[b], msk.data_ptr(), params[s], mout, mdst[s & 1].data_ptr(), stream)
            return
        ctx.pair_batch(idescs[b], img.data_ptr(), mdescs[b], msk.data_ptr(), params[s], iout, idst[s & 1].data_ptr(),
                       mout, mdst[s & 1].data_ptr(), stream)

    for s in range(warmup):
        step(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(warmup, warmup + steps):
        step(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"value": batch * steps / dt, "unit": "images/s (image+mask pairs)", "batch": batch,
           "ms_per_step": dt / steps * 1e3, "source": f"{w}x{h} u8 HWC image + {w}x{h} u8 mask",
           "what": "image 512x512x3 f32 CHW (bilinear) + mask 512x512 u8 (nearest), shared params, one "
                   "aeon_hip_augment_pair_batch call per batch"}
    if not kernel_timing:
        ctx.close()
        return res
    # kernel durations: the same steps again with every launch timed (the events cost GPU time
    # between launches, so the rate above is taken without them)
    ctx.kernel_times()
    ctx.set_timing(1)
    for s in range(warmup, warmup + steps):
        step(s)
    ctx.synchronize(stream)
    k_ms, k_bytes, k_n = ctx.kernel_times()["augment"]
    ctx.set_timing(False)
    ctx.close()
    res.update(kernels_ms_per_step=k_ms / steps, kernels_gbs=k_bytes / (k_ms * 1e-3) / 1e9 if k_ms else 0)
    return res


def pool_threads():
    """aeon's decode pool size, hc - min(2, hc/8) (src/util.cpp:360-370), over the CPUs this
    process may use (OMP_NUM_THREADS on the GPU box, else the affinity mask)."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    hc = int(os.environ.get("OMP_NUM_THREADS") or visible)
    return max(1, hc - min(2, hc // 8)), hc, visible


def pin_baseline(A):
    """The CPU baseline's pool pinned like aeon's decode pool: worker t on CPU t of the product's
    thread_affinity_map (AEON_CPU_LIST, else aeon's hc - min(2, hc/8) policy over this process's CPUs)."""
    import oracle as O
    _, hc, visible = pool_threads()
    cpus = A.thread_affinity_map()
    O.set_affinity(cpus)
    return len(cpus), hc, visible, cpus


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(A, C, budget_s, cfg="C2"):
    """aeon's CPU path restated (oracle/, C++): a pool of hc - min(2, hc/8) workers with a
    dynamic atomic task counter (src/util.cpp:360-370, src/thread_pool.hpp:155-162) over
    decode windows of the config's batch.  Scalar C++ with -ffp-contract=off, not OpenCV's SIMD
    paths: a LOWER BOUND on aeon's own CPU rate."""
    import numpy as np
    import oracle as O
    from tests import helpers as H
    threads, hc, visible, cpus = pin_baseline(A)
    if cfg == "C5":
        n, w, h = 128, 640, 480
        imgs = [A.synthetic_image(i, w, h, 3) for i in range(n)]
        rng = np.random.default_rng(5)
        masks = [rng.integers(0, 21, (h, w), dtype=np.uint8) for _ in range(n)]
        params = H.draw_params(C.C5_AUG, [(w, h)] * n, 512, 512, seed=1)
        lc = H.oracle_load_config(C.out_desc_for(C.IMAGE_512, C.C5_AUG))
        mlc = H.oracle_load_config(C.out_desc_for(C.MASK_512, C.C5_AUG))
        q = [H.to_oracle_params(p) for p in params]
        run = lambda: O.batch_image_mask(imgs, masks, q, lc, (3, 512, 512), mlc, (1, 512, 512), threads)[2]
        what = f"C5 image+mask pairs, {w}x{h} -> 512x512"
    else:
        aug = {"C1": C.C1_AUG, "C2": C.C2_AUG, "C3": C.C3_AUG}[cfg]
        # C1 = aeon's own eval config on decoded images of its golden record's size (480x360), in
        # aeon's decode_size windows (batch 32 -> the smallest multiple giving each thread 8 records,
        # src/loader.cpp:162-164); C2 / C3 in 256-record windows
        n, w, h = {"C1": (32 * ((threads * 8 - 1) // 32 + 1), 480, 360), "C2": (256, 256, 256),
                   "C3": (256, 256, 256)}[cfg]
        imgs = [A.synthetic_image(i, w, h, 3) for i in range(n)]
        params = H.draw_params(aug, [(w, h)] * n, 224, 224, seed=1)
        lc = H.oracle_load_config(C.out_desc_for(C.IMAGE_224, aug))
        q = [H.to_oracle_params(p) for p in params]
        run = lambda: O.batch_augment(imgs, q, lc, (3, 224, 224), threads)[1]
        what = f"{cfg} on {w}x{h} records -> 224x224 fp32 CHW"
    done, secs = 0, 0.0
    while secs < budget_s:
        secs += run()
        done += n
    return {"value": done / secs, "unit": "images/s" if cfg != "C5" else "image+mask pairs/s", "cores": threads,
            "kind": "port",
            "sample": f"{what}: {done} records in windows of {n} ({secs:.1f} s CPU wall); oracle/ C++ restatement "
                      f"of aeon's transform+load on {threads} pool threads pinned one per CPU to "
                      f"[{cpu_list_str(cpus)}] (aeon's thread_affinity_map over {hc} usable CPUs; "
                      f"{visible} in the affinity mask, {os.cpu_count()} on the machine; CPU: {cpu_model()}); "
                      "scalar C++, a lower bound on aeon's OpenCV-SIMD path"}


def run_aeon_path(A, C, torch, cfg="C2", overlap=True, windows=8, warmup=2):
    """aeon's own decode stage with the HIP stager in place of provide()'s pixel work, emulated call for
    call (INTEGRATION.md edits 1-4; tests/test_integration.py checks the same sequence bit-exact): a
    decode thread runs provide() for a window of decoded records on 8 pool threads (make_params +
    aeon_hip_stager_stage; the params drawn before the timed windows) and post_process() per batch; the consumer (batch_iterator_fbm::filler) takes
    the batches out of the container -- two containers alternate (async_manager).  overlap=True:
    post_process is launch-only and the consumer waits per buffer (edits 3 + 4), so window k's GPU work
    runs while window k+1 is staged; False: post_process flushes (launch + wait).  Pageable host batch
    buffers (aeon's default: the stager copies each batch back with a D2H).  Records/s over `windows`."""
    import queue
    import threading
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    aug = {"C1": C.C1_AUG, "C2": C.C2_AUG}[cfg]
    batch, nb = (32, 4) if cfg == "C1" else (64, 4)
    src_w, src_h = (480, 360) if cfg == "C1" else (256, 256)
    n = batch * nb
    ctx = A.Context(torch.cuda.current_device())
    out = C.out_desc_for(C.IMAGE_224, aug)
    st = A.Stager(ctx, out, batch)
    factory = A.ParamFactory(aug)
    engines = A.seed_slots(1, n)
    recs = [A.synthetic_image(i, src_w, src_h, 3) for i in range(n)]
    conts = [[np.zeros(batch * out.item_stride, np.uint8) for _ in range(nb)] for _ in range(2)]
    total = warmup + windows
    # the windows' params drawn up front (aeon draws them inside provide(), natively, ~1.5 us per
    # record; drawn here they would measure the Python interpreter instead)
    params = []
    for _ in range(total):
        params.append([factory.make_params(engines[i:i + 1], src_w, src_h, 224, 224) for i in range(n)])
    free_q, full_q = queue.Queue(), queue.Queue()
    for c in range(2):
        free_q.put(c)
    t_start = [0.0]

    def decode_stage():
        with ThreadPoolExecutor(max_workers=8) as pool:
            for w in range(total):
                c = free_q.get()
                if w == warmup:
                    t_start[0] = time.perf_counter()

                def provide(b):  # one batch's records per task (the stage copies run without the GIL)
                    for i in range(b * batch, (b + 1) * batch):
                        st.stage(conts[c][b].ctypes.data, i % batch, recs[i], params[w][i])

                list(pool.map(provide, range(nb)))
                for b in range(nb):
                    (st.launch if overlap else st.flush)(conts[c][b].ctypes.data)
                full_q.put(c)

    th = threading.Thread(target=decode_stage)
    th.start()
    sink = 0
    for w in range(total):
        c = full_q.get(timeout=300)
        for b in range(nb):
            A.Stager.wait_buffer(conts[c][b].ctypes.data)  # (flush mode: returns at once)
            sink += int(conts[c][b][0])  # the consumer touches the batch
        free_q.put(c)
    dt = time.perf_counter() - t_start[0]
    th.join()
    st.close()
    ctx.close()
    return {"value": n * windows / dt, "unit": "images/s", "batch": batch, "decode_size": n,
            "ms_per_window": dt / windows * 1e3}


def run_aeon_path_cpp(windows=24, warmup=4, reps=2):
    """aeon's decode stage with the stager, call for call, as a C++ program against the C ABI
    (tools/aeon_path_cpp.cpp, built as aeon_amd/aeon_path_cpp; INTEGRATION.md edits 1-5): aeon's pinned pool of
    thread_affinity_map workers running provide() (make_params from each record's slot engine +
    aeon_hip_stager_stage of a decoded host record) over aeon's decode_size window, post_process() per batch,
    a consumer thread waiting per buffer over two alternating containers.  Per config, batch buffers pageable
    or pinned ("pinned": true -> aeon_hip_host_alloc, the kernels store into them), post_process launch-only
    with the consumer's wait ('overlap') or flushing; each run `reps` times (the host's load swings these
    PCIe/host-bound rates), all values kept, best first."""
    import subprocess
    exe = os.path.join(ROOT, "aeon_amd", "aeon_path_cpp")
    res = {}
    for cfg in ("C2", "C1"):
        for buffers in ("pinned", "pageable"):
            for mode in ("overlap", "flush"):
                vals = []
                for _ in range(reps):
                    r = subprocess.run([exe, cfg, buffers, mode, str(windows), str(warmup)], capture_output=True,
                                       text=True, timeout=180)
                    if r.returncode != 0:
                        raise RuntimeError(f"aeon_path_cpp {cfg} {buffers} {mode}: {r.stderr.strip()[-300:]}")
                    vals.append(json.loads(r.stdout.strip().splitlines()[-1]))
                vals.sort(key=lambda d: -d["value"])
                res.setdefault(cfg, {}).setdefault(buffers, {})[mode] = {
                    "value": vals[0]["value"], "runs": [round(v["value"]) for v in vals], "unit": "images/s",
                    "batch": vals[0]["batch"], "decode_size": vals[0]["decode_size"],
                    "pool_threads": vals[0]["pool_threads"]}
    res["what"] = ("tools/aeon_path_cpp.cpp: aeon's decode stage in C++ (loader.cpp:158-176 pool and decode_size, "
                   "batch_decoder::filler's provide + post_process, batch_iterator_fbm::filler's wait, two containers)")
    return res


def side(extra, key, fn):
    """One side run of the bench line (rank 0's extras): a failure is recorded in the line under its
    key instead of losing the line."""
    try:
        extra[key] = fn()
    except Exception as e:  # noqa: BLE001 -- any failure of a side run
        extra[key] = {"error": f"{type(e).__name__}: {e}"}


def jpeg_files(batch):
    """Encoded records of a decode window: aeon's own JPEG fixtures (test/test_data/img_2112_70.jpg
    480x360 and flowers.jpg 600x800, 4:2:0 baseline; committed in tests/golden), cycled."""
    import numpy as np
    fx = np.load(os.path.join(ROOT, "tests", "golden", "jpeg_fixtures.npz"))
    files = [fx["img_2112_70.jpg"].tobytes(), fx["flowers.jpg"].tobytes()]
    return [files[i % 2] for i in range(batch)]


def run_e2e_jpeg(A, C, torch, batch=512, windows=30, on_device=False):
    """The product's whole decode stage from encoded records, double-buffered (aeon_decoder_submit /
    wait over two windows): JPEG entropy decode on the host pool, sparse coefficients H2D, GPU IDCT
    + colour into the source arena, C2 augmentation, and (host outputs) D2H into pinned buffers."""
    cfg = dict(C.CONFIGS["C2"], random_seed=1)
    files = jpeg_files(batch)
    d = A.Decoder(cfg)
    recs = d.encoded([(f,) for f in files])  # (marshalled once: aeon's host hands over plain pointers)
    item = 3 * 224 * 224 * 4
    if on_device:
        bufs = [torch.empty(batch * item, dtype=torch.uint8, device="cuda") for _ in range(2)]
    else:
        bufs = [torch.empty(batch * item, dtype=torch.uint8).pin_memory() for _ in range(2)]
    for w in range(2):  # warmup: contexts, staging, kernels
        d.submit(recs, [bufs[w].data_ptr()], on_device)
    d.wait()
    d.wait()
    t0 = time.perf_counter()
    for w in range(windows):
        if w >= 2:
            d.wait()
        d.submit(recs, [bufs[w % 2].data_ptr()], on_device)
    d.wait()
    d.wait()
    dt = time.perf_counter() - t0
    d.close()
    return batch * windows / dt


def run_jpeg_stage(A, torch, batch=512, reps=60):
    """aeon_hip_decode_jpeg_batch alone (extract of a window of JPEG files into device memory): a
    512-record window (aeon's decode_size = 2 x batch 256), so the GPU Huffman decoder holds two files per
    CU."""
    files = jpeg_files(batch)
    ctx = A.Context(torch.cuda.current_device())
    infos = [A.jpeg_info(f) for f in files]
    descs, off = [], 0
    for (w, h, _) in infos:
        descs.append(A.ImgDesc(offset=off, width=w, height=h, stride=w * 3, channels=3))
        off += (w * h * 3 + 15) // 16 * 16
    descs = (A.ImgDesc * batch)(*descs)
    dst = torch.empty(off, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream().cuda_stream  # (a stream of our own: see run_device)
    jf = A.JpegFiles(files)  # (marshalled once: aeon's host hands over plain pointers)
    # warmup: both staging sets allocated (their first use grows pinned buffers), the pool's threads and
    # caches warm (20 timed calls right after two warmups read 84-243 K on one box)
    for _ in range(8):
        ctx.decode_jpeg_batch(jf, descs, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.decode_jpeg_batch(jf, descs, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    dt = time.perf_counter() - t0
    # the GPU part alone: HIP events around the IDCT + colour launches of every call
    ctx.kernel_times()
    ctx.set_timing(1)
    for _ in range(reps):
        ctx.decode_jpeg_batch(jf, descs, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    k_ms, k_px, k_n = ctx.kernel_times()["jpeg"]
    ctx.set_timing(False)
    ctx.close()
    # the host part alone, per distinct file on this thread: what the stage does on the pool (headers
    # + unstuffed entropy-coded bytes for the GPU decoder) and, for reference, a host Huffman decode
    host_us, huff_us = {}, {}
    for name, f in (("img_2112_70.jpg", files[0]), ("flowers.jpg", files[1])):
        for fn, out in ((A.jpeg_host_stage, host_us), (A.jpeg_entropy_decode, huff_us)):
            t1 = time.perf_counter()
            for _ in range(20):
                fn(f)
            out[name] = (time.perf_counter() - t1) / 20 * 1e6
    mp = sum(w * h for (w, h, _) in infos) / batch / 1e6
    gpu_entropy = all(A.jpeg_host_stage(f)[0] for f in files[:2])
    return {"value": batch * reps / dt, "unit": "images/s", "megapixels_per_image": mp,
            "gpu_us_per_record": k_ms * 1e3 / max(k_n, 1) / batch if k_n else None,
            "gpu_kernel_gbs": k_px / (k_ms * 1e-3) / 1e9 if k_ms else None,
            "host_stage_us_per_file": host_us, "host_huffman_us_per_file": huff_us,
            "entropy_decoding": "gpu" if gpu_entropy and os.environ.get("AEON_HIP_JPEG_HUFF") != "host" else "host",
            "what": "aeon_hip_decode_jpeg_batch: headers on the pool, entropy-coded bytes H2D, GPU Huffman "
                    "decode (jpeg_huff) + ISLOW IDCT + fancy upsampling + YCbCr->BGR into device memory; "
                    "gpu_us_per_record covers the three kernels"}


def cpu_baseline_jpeg(A, C, budget_s):
    """aeon's full CPU path per record (imdecode -> transform -> load) restated by the oracle, on the
    same encoded files and C2 params, aeon's pool policy: a lower bound (scalar decode, no SIMD)."""
    import oracle as O
    from tests import helpers as H
    threads, hc, visible, cpus = pin_baseline(A)
    files = jpeg_files(256)
    sizes = [O.jpeg_info(f)[:2] for f in files]
    params = [H.to_oracle_params(p) for p in H.draw_params(C.C2_AUG, sizes, 224, 224, seed=1)]
    lc = H.oracle_load_config(C.out_desc_for(C.IMAGE_224, C.C2_AUG))
    done, secs = 0, 0.0
    while secs < budget_s:
        secs += O.batch_decode_augment(files, params, lc, (3, 224, 224), threads)[1]
        done += len(files)
    return {"value": done / secs, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{done} JPEG records (img_2112_70.jpg / flowers.jpg) decoded + C2-augmented by the oracle "
                      f"on {threads} pool threads pinned to [{cpu_list_str(cpus)}] ({secs:.1f} s); scalar C++, "
                      "a lower bound on aeon's "
                      "libjpeg-turbo + OpenCV-SIMD path"}


def run_c1_decoder(A, C, torch, budget_s=2.0):
    """C1 through the product's decode stage (aeon_decoder: provider_factory + batch_decoder,
    host records in, host batch out): decode windows of 480x360 decoded records, two windows in
    flight (submit / wait) into pinned host batches.  The window is aeon's decode_size, the smallest
    multiple of batch_size giving every pool thread 8 records (src/loader.cpp:162-164,
    m_input_multiplier src/loader.hpp:237): 128 records for batch 32 on 14 threads."""
    cfg = dict(C.CONFIGS["C1"], random_seed=1)
    d = A.Decoder(cfg)
    batch = cfg["batch_size"]
    threads = len(A.thread_affinity_map())
    n = batch * ((threads * 8 - 1) // batch + 1)
    recs = [(A.synthetic_image(i, 480, 360, 3),) for i in range(n)]
    bufs = [torch.empty(n * 3 * 224 * 224 * 4, dtype=torch.uint8).pin_memory() for _ in range(2)]
    for w in range(2):  # warmup (context, kernels, buffers)
        d.submit(recs, [bufs[w].data_ptr()])
    d.wait()
    d.wait()
    done, w, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        if w >= 2:
            d.wait()
        d.submit(recs, [bufs[w % 2].data_ptr()])
        w += 1
        done += n
    d.wait()
    d.wait()
    dt = time.perf_counter() - t0
    d.close()
    return {"value": done / dt, "unit": "images/s", "batch": batch, "decode_size": n,
            "what": "aeon_decoder submit/wait: host decoded 480x360 records -> pinned H2D -> resize_short 256 + "
                    f"center crop 224 -> fp32 CHW -> D2H into pinned batches, two {n}-record windows (aeon's "
                    "decode_size) in flight"}


def load_traffic(path, cfg):
    try:
        d = json.load(open(path))
        return d.get(cfg, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def dry_run(args, world, rank):
    """CPU rehearsal of the N-rank path with gloo: every rank takes its aeon node slice and decoder
    seed, draws its first window of params, and times stub steps; rank 0 prints the line with each
    rank's slice head / length and slot states, and the max-over-ranks time."""
    import torch
    import torch.distributed as dist
    import aeon_amd as A
    from aeon_amd import configs as C
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    batch = args.batch or C.CONFIGS[args.config]["batch_size"]
    n_records = 16 * batch * world
    records, seed = rank_slice(n_records, batch, rank, world)
    states = A.seed_slots(seed, 4)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.0005)
    elapsed = time.perf_counter() - t0
    cpus = rank_cpu_lists([None] * world, set(os.sched_getaffinity(0)), world)[rank]
    mine = {"rank": rank, "node_id": rank, "seed": seed, "slice_len": len(records),
            "slice_head": [int(x) for x in records[:2 * batch]], "slot_states": [int(x) for x in states],
            "cpu_list": cpu_list_str(cpus)}
    allv = [None] * world
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.all_gather_object(allv, mine)
        dist.destroy_process_group()
    else:
        allv = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "steps": args.steps, "batch_per_rank": batch,
                          "n_records": n_records, "elapsed_max_s": elapsed, "ranks": allv}), flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import aeon_amd as A
    from aeon_amd import configs as C

    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.share_device:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    batch = args.batch or C.CONFIGS[args.config]["batch_size"]
    cpu_lists = None
    if world > 1:
        # one process per GPU: every rank's decode pools (aeon_decoder, the JPEG stage) pinned to its own
        # block of its GPU's NUMA-local CPUs (AEON_CPU_LIST, util.cpp:344-357), no two ranks sharing one
        ngpu = torch.cuda.device_count()
        local_sets = [gpu_local_cpus(torch, (r % ngpu) if args.share_device else r) for r in range(world)]
        cpu_lists = rank_cpu_lists(local_sets, set(os.sched_getaffinity(0)), world)
        os.environ["AEON_CPU_LIST"] = cpu_list_str(cpu_lists[rank])

    # C2 (one launch per step): the region event pair; C3 (two passes and a reduce per step): sampled
    # per-launch events, one step in ten unless --timing-every says otherwise
    region = args.config == "C2" and args.streams == 1
    timing = args.timing_every or (0 if region else 10)
    elapsed, kt, param_us, submit_s = run_device(A, C, torch, args.config, batch, args.steps, args.warmup,
                                                 rank, world, args.pool_mib, dist, timing, args.streams,
                                                 region=region)
    total = batch * args.steps * world
    value = total / elapsed
    k_ms, k_bytes, k_n = kt["augment"]
    # dominant kernel = augment_tiles<KM_FINAL,...>: algorithmic bytes per launch / its average
    # launch duration (one HIP event pair on the launch stream around the timed region's launches
    # 2..K, back to back: run_device(region=True); one launch per C2 step)
    achieved = k_bytes / (k_ms * 1e-3) / 1e9 if k_ms else 0.0
    bytes_per_launch = k_bytes / max(k_n, 1)

    extra = {}
    if world > 1 and not args.no_extra:
        # C4 (BASELINE configs[3]): the full augment_image workload at per-GPU batch 1024 on every
        # rank, each its own node slice and seed; global batch 1024 * N
        # (the rate from an untimed run -- an event pair around a launch idles the queue around it --
        # the kernel duration from a second, short run that times every launch, as the C3 extra does)
        st4 = max(5, args.steps // 5)
        e4, _, _, _ = run_device(A, C, torch, "C3", 1024, st4, 2, rank, world, args.pool_mib, dist, 0)
        _, kt4, _, _ = run_device(A, C, torch, "C3", 1024, 4, 1, rank, world, args.pool_mib, dist, 1)
        m4, b4, n4 = kt4["augment"]
        extra["C4"] = {"value": 1024 * st4 * world / e4, "unit": "images/s", "batch_per_gpu": 1024,
                       "global_batch": 1024 * world, "steps": st4, "ms_per_step": e4 / st4 * 1e3,
                       "augment_kernel_avg_launch_ms": m4 / max(n4, 1),
                       "what": "C3 workload on every rank (node slice + seed 1 + node_id), max over ranks; "
                               "rate untimed, kernel time from a second run timing every launch"}
    if rank == 0 and world == 1 and not args.no_extra:
        if args.config == "C2":
            # rate untimed (an event pair between a step's launches costs ~10 us of GPU time there),
            # the kernel durations from a second run timing every launch
            def c3():
                st3 = max(30, args.steps)
                e3, _, _, _ = run_device(A, C, torch, "C3", 1024, st3, 3, 0, 1, args.pool_mib, None, 0)
                _, kt3, _, _ = run_device(A, C, torch, "C3", 1024, 6, 2, 0, 1, args.pool_mib, None, 1)
                m3, b3, n3 = kt3["augment"]
                s3 = kt3["stats"]
                # consecutive batches alternating over two streams (aeon_decoder's two windows): a CU
                # that finishes its last record starts the next launch's first while the others drain
                e32, _, _, _ = run_device(A, C, torch, "C3", 1024, st3, 3, 0, 1, args.pool_mib, None, 0, 2)
                return {"value": 1024 * st3 / e3, "unit": "images/s", "batch": 1024,
                        "ms_per_step": e3 / st3 * 1e3,
                        "two_streams": {"value": 1024 * st3 / e32, "ms_per_step": e32 / st3 * 1e3},
                        "augment_kernel_avg_launch_ms": m3 / max(n3, 1),
                        "stats_kernel_avg_launch_ms": s3[0] / max(s3[2], 1),
                        "augment_kernel_gbs": b3 / (m3 * 1e-3) / 1e9 if m3 else 0}
            side(extra, "C3", c3)
        if args.streams == 1:
            # the same C2 steps alternating over two caller streams (one per output container,
            # as aeon's double-buffered async_manager holds two batches): the next batch's launch
            # is dispatched while the current one drains, hiding the ~6 us dispatch gap
            def two_streams():
                e2, _, _, _ = run_device(A, C, torch, args.config, batch, args.steps, args.warmup, 0, 1,
                                         args.pool_mib, None, 0, 2)
                return {"value": batch * args.steps / e2, "unit": "images/s", "ms_per_step": e2 / args.steps * 1e3,
                        "what": "same workload, consecutive batches on two streams"}
            side(extra, "two_streams", two_streams)
        side(extra, "C5", lambda: run_c5(A, C, torch, max(20, args.steps), 3, args.pool_mib))

        # aeon's other interpolation methods on the C2 workload: CUBIC / LANCZOS4 / AREA as resize_sep bands
        # (AREA: its resizeArea_ form and the bilinear emulation), writing the loader's f32 CHW output themselves (no photometric
        # stage in C2); the rate from an untimed run, each kernel kind's time, bytes and HBM fraction
        # from a second run with every launch timed
        def interpolation():
            out = {}
            for m in ("CUBIC", "AREA", "LANCZOS4"):
                # (10 warmup calls: LANCZOS4's per-thread sin / cos memo warms over the plan pool's threads)
                em, _, _, _ = run_device(A, C, torch, "C2:" + m, batch, 20, 10, 0, 1, args.pool_mib, None, 0)
                _, ktm, _, _ = run_device(A, C, torch, "C2:" + m, batch, 20, 3, 0, 1, args.pool_mib, None, 1)
                kinds = {}
                for k, (ms, by, n) in ktm.items():
                    if n and ms > 0:
                        gbs = by / (ms * 1e-3) / 1e9
                        kinds[k] = {"us_per_step": ms / 20 * 1e3, "algorithmic_bytes_per_step": by / 20,
                                    "gbs": gbs, "roofline_frac": gbs / HBM_PEAK_GBS}
                out[m] = {"value": batch * 20 / em, "unit": "images/s", "ms_per_step": em / 20 * 1e3, "kernels": kinds}
            out["what"] = ("C2 workload (batch 256) with interpolation_method set: value from an untimed run; "
                           "kernels: 'pre' = the resize pass (resize_sep bands, f32 CHW output), 'augment' = "
                           "tile launches of records the resize pass does not take; every launch timed there")
            return out
        side(extra, "interpolation", interpolation)
        side(extra, "e2e_host_to_host", lambda: {
            "value": run_e2e(A, C, torch, 256, 20), "unit": "images/s",
            "what": "pinned H2D of decoded 256x256 u8 + kernel + D2H of fp32 CHW"})
        side(extra, "e2e_zero_copy", lambda: {
            "value": run_e2e(A, C, torch, 256, 20, zero_copy=True), "unit": "images/s",
            "what": "pinned H2D of decoded 256x256 u8 + kernel storing fp32 CHW straight into the pinned host "
                    "batch (zero-copy over PCIe, no D2H)"})
        side(extra, "C1", lambda: {"decoder": run_c1_decoder(A, C, torch)})

        side(extra, "aeon_path_cpp", run_aeon_path_cpp)
        side(extra, "e2e_jpeg_decoder", lambda: {
            "host_outputs": {"value": run_e2e_jpeg(A, C, torch, on_device=False), "unit": "images/s"},
            "device_outputs": {"value": run_e2e_jpeg(A, C, torch, on_device=True), "unit": "images/s"},
            "jpeg_stage": run_jpeg_stage(A, torch),
            "what": "encoded JPEG records (aeon's img_2112_70.jpg / flowers.jpg) -> aeon_decoder submit/wait "
                    "(two windows in flight): extract on the JPEG stage + C2 augmentation, 512-record windows "
                    "(decode_size = 2 x batch 256)"})
        if not args.no_cpu_baseline:
            for key, fn in (("e2e_jpeg_decoder", lambda: cpu_baseline_jpeg(A, C, args.cpu_extra_seconds)),
                            ("C1", lambda: cpu_baseline(A, C, args.cpu_extra_seconds, "C1")),
                            ("C3", lambda: cpu_baseline(A, C, args.cpu_extra_seconds, "C3")),
                            ("C5", lambda: cpu_baseline(A, C, args.cpu_extra_seconds, "C5"))):
                if isinstance(extra.get(key), dict) and "error" not in extra[key]:
                    side(extra[key], "cpu_baseline", fn)

    line = {
        "metric": METRIC,
        "value": value,
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        # integer pixel arithmetic (u8 fixed-point resize / photometric), f32 only in the final
        # standardize of the 3x224x224 float32 CHW output
        "dtype": "u8",
        "data": "synthetic: A.synthetic_image (splitmix64) HWC u8 256x256 sources of this rank's manifest "
                "slice, resident in HBM",
        "config": {"workload": f"{args.config}: " + {
            "C2": "random crop + flip + bilinear resize to 224x224, standardize, CHW fp32",
            "C3": "full augment_image (brightness/contrast/saturation/hue/lighting), CHW fp32"}[args.config],
            "batch_per_gpu": batch, "global_batch": batch * world, "source": "256x256x3 u8 HWC",
            "output": "3x224x224 float32 CHW",
            "parallelism": f"dp{world}: one aeon manifest node slice + seed per rank, no collective"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_traffic(args.traffic_file, args.config),
                     "kernel": "augment_tiles<KM_FINAL,...>", "kernel_avg_launch_ms": k_ms / max(k_n, 1),
                     "algorithmic_bytes_per_launch": bytes_per_launch, "timed_launches": k_n,
                     "timing": "one HIP event pair on the launch stream around launches 2..K of the timed region "
                               "(back to back, as rocprofv3 sees them)",
                     # the same algorithmic bytes over the whole step (upload + kernel + host)
                     "step_gbs": bytes_per_launch / (elapsed / args.steps) / 1e9 if k_n else None},
        "host_make_params_us_per_record": param_us,
        "decode_pool_cpus": ({str(r): cpu_list_str(l) for r, l in enumerate(cpu_lists)} if cpu_lists else
                             cpu_list_str(A.thread_affinity_map())),
        "host_submit_ms_per_step": submit_s / args.steps * 1e3,
    }
    if extra:
        line["extra"] = extra
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(A, C, args.cpu_seconds, args.config)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
