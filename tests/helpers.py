"""Shared helpers: run the same records through the HIP stage and through the CPU oracle."""
import numpy as np

import aeon_amd as A
import oracle as O


def oracle_aug_config(aug):
    """aeon augmentation JSON -> oracle AugConfig (the checker's own plain struct)."""
    kw = {}
    for key, lo, hi in (("scale", "scale_min", "scale_max"),
                        ("horizontal_distortion", "hdist_min", "hdist_max"),
                        ("contrast", "contrast_min", "contrast_max"),
                        ("brightness", "brightness_min", "brightness_max"),
                        ("saturation", "saturation_min", "saturation_max")):
        if key in aug:
            kw[lo], kw[hi] = aug[key]
    if "angle" in aug:
        kw["angle_min"], kw["angle_max"] = aug["angle"]
    if "hue" in aug:
        kw["hue_min"], kw["hue_max"] = aug["hue"]
    if "lighting" in aug:
        kw["lighting_mean"], kw["lighting_stddev"] = aug["lighting"]
    for key in ("flip_enable", "center", "crop_enable", "do_area_scale"):
        if key in aug:
            kw[key] = int(aug[key])
    for key in ("resize_short_size", "padding"):
        if key in aug:
            kw[key] = aug[key]
    if "fixed_scaling_factor" in aug:
        kw["fixed_scaling_factor"] = aug["fixed_scaling_factor"]
    kw["interp"] = O.INTERP[aug.get("interpolation_method", "LINEAR").upper()]
    if "expand_ratio" in aug:
        kw["expand_ratio_min"], kw["expand_ratio_max"] = aug["expand_ratio"]
    if "expand_probability" in aug:
        kw["expand_probability"] = aug["expand_probability"]
    samplers = []
    for bs in aug.get("batch_samplers", []):
        bs = bs or {}
        sm, sc = bs.get("sampler") or {}, bs.get("sample_constraint") or {}
        samplers.append(O.batch_sampler(max_sample=bs.get("max_sample", -1), max_trials=bs.get("max_trials", 100),
                                        scale=tuple(sm.get("scale", (1.0, 1.0))),
                                        aspect_ratio=tuple(sm.get("aspect_ratio", (1.0, 1.0))),
                                        **{k + "_" + v: sc[k + "_" + w] for k in ("min", "max")
                                           for v, w in (("jaccard", "jaccard_overlap"), ("sample_cov", "sample_coverage"),
                                                        ("object_cov", "object_coverage"))
                                           if k + "_" + w in sc}))
    if samplers:
        kw["samplers"] = samplers
    return O.aug_config(**kw)


def oracle_load_config(out):
    """aeon_amd.OutDesc -> oracle LoadConfig."""
    name = {code: n for n, (code, _) in A.DTYPES.items()}[out.dtype]
    return O.load_config(out.channels, bool(out.channel_major), bool(out.bgr_to_rgb), name,
                         list(out.mean) if out.has_mean else None,
                         list(out.stddev) if out.has_mean else None)


def to_oracle_params(p):
    q = O.Params()
    for f, _ in O.Params._fields_:
        if f == "lighting":
            for i in range(3):
                q.lighting[i] = p.lighting[i]
        else:
            setattr(q, f, getattr(p, f))
    return q


def oracle_records(images, params, out, mask=False):
    lc = oracle_load_config(out)
    res = []
    for im, p in zip(images, params):
        q = to_oracle_params(p)
        if mask:
            m = O.transform_mask(im, q)
            res.append(O.load_image(m[:, :, None], lc))
        else:
            res.append(O.augment_record(im, q, lc))
    return res


def place_canvas(rec, out):
    """image::loader with fixed_aspect_ratio (aeon src/etl_image.cpp:258-306): a zeroed
    canvas_w x canvas_h canvas with the record at its top-left (uint8 output)."""
    cn = out.channels
    if out.channel_major:
        c = np.zeros((cn, out.canvas_h, out.canvas_w), np.uint8)
        c[:, :rec.shape[1], :rec.shape[2]] = rec
    else:
        c = np.zeros((out.canvas_h, out.canvas_w, cn), np.uint8)
        c[:rec.shape[0], :rec.shape[1], :] = rec
    return c


def hip_canvases(ctx, images, params, out, mask=False):
    """fixed_aspect_ratio: the whole canvas of every item (the output buffer starts as 0xAB so
    the zero fill is checked too)."""
    import torch
    arena, descs = A.pack_images(images)
    src = torch.from_numpy(arena).to("cuda")
    n = len(images)
    dst = torch.full((n * out.item_stride,), 0xAB, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    (ctx.mask_batch if mask else ctx.augment_batch)(descs, src.data_ptr(), params, out, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    host = dst.cpu().numpy()
    cn = out.channels
    shape = (cn, out.canvas_h, out.canvas_w) if out.channel_major else (out.canvas_h, out.canvas_w, cn)
    nb = int(np.prod(shape))
    return [host[i * out.item_stride: i * out.item_stride + nb].reshape(shape).copy() for i in range(n)]


def hip_records(ctx, images, params, out, mask=False, dtype=None, info=None):
    """Run records through the HIP stage on cuda:0; returns one array per record.  info (a dict): gets
    the device output buffer's address ('dst_ptr') for failure reports."""
    import torch
    arena, descs = A.pack_images(images)
    src = torch.from_numpy(arena).to("cuda") if arena.size else torch.zeros(16, dtype=torch.uint8, device="cuda")
    n = len(images)
    dst = torch.zeros(max(n, 1) * out.item_stride, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    fn = ctx.mask_batch if mask else ctx.augment_batch
    fn(descs, src.data_ptr(), params, out, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    if info is not None:
        info["dst_ptr"] = dst.data_ptr()
    host = dst.cpu().numpy()
    res = []
    for i, p in enumerate(params):
        cn = out.channels
        shape = (cn, p.out_h, p.out_w) if out.channel_major else (p.out_h, p.out_w, cn)
        dt = A.NP_DTYPE[out.dtype]
        nbytes = int(np.prod(shape)) * np.dtype(dt).itemsize
        item = host[i * out.item_stride: i * out.item_stride + nbytes].view(dt).reshape(shape)
        res.append(item.copy())
    return res


def draw_params(aug, sizes, out_w, out_h, seed=1):
    """make_params per record with aeon deterministic-mode slot engines (one per record)."""
    f = A.ParamFactory(aug)
    states = A.seed_slots(seed, len(sizes))
    res = []
    for i, (w, h) in enumerate(sizes):
        st = states[i:i + 1].copy()
        res.append(f.make_params(st, w, h, out_w, out_h))
    return res


def lost_lines_report(dst_ptr, item_stride, index, got, want):
    """Where a device output differs from the oracle: the 128-byte lines' device addresses and whether
    each lies inside one of the process's uncached job-table blocks (A.uncached_blocks), with the
    blocks' ranges -- the evidence the lost-line fault of DESIGN.md §8 needs."""
    g = np.ascontiguousarray(got).view(np.uint8).reshape(-1)
    w = np.ascontiguousarray(want).view(np.uint8).reshape(-1)
    off = np.nonzero(g != w)[0]
    if not off.size:
        return "no difference"
    base = dst_ptr + index * item_stride
    lines = sorted({(base + int(o)) & ~127 for o in off})
    blocks = A.uncached_blocks()
    inside = [ln for ln in lines if any(lo <= ln < hi for lo, hi in blocks)]
    return (f"record {index}: {off.size} bytes differ in {len(lines)} lines of 128 B at device "
            f"{hex(lines[0])}..{hex(lines[-1])} (buffer {hex(dst_ptr)}); {len(inside)} of them inside an uncached "
            f"job-table block; blocks: {[(hex(lo), hex(hi)) for lo, hi in blocks]}")
