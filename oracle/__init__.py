"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  It is the checker, never the product: aeon_amd/ does not import it.
See aeon_oracle.h for what is restated and which reference lines each part follows.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class BatchSampler(ctypes.Structure):
    _fields_ = [("max_sample", ctypes.c_int), ("max_trials", ctypes.c_int),
                ("scale_min", ctypes.c_float), ("scale_max", ctypes.c_float),
                ("ar_min", ctypes.c_float), ("ar_max", ctypes.c_float),
                ("min_jaccard", ctypes.c_float), ("max_jaccard", ctypes.c_float),
                ("min_sample_cov", ctypes.c_float), ("max_sample_cov", ctypes.c_float),
                ("min_object_cov", ctypes.c_float), ("max_object_cov", ctypes.c_float)]


def batch_sampler(max_sample=-1, max_trials=100, scale=(1.0, 1.0), aspect_ratio=(1.0, 1.0), **constraint):
    nan = float("nan")
    b = BatchSampler(max_sample=max_sample, max_trials=max_trials, scale_min=scale[0], scale_max=scale[1],
                     ar_min=aspect_ratio[0], ar_max=aspect_ratio[1])
    for k in ("min_jaccard", "max_jaccard", "min_sample_cov", "max_sample_cov", "min_object_cov", "max_object_cov"):
        setattr(b, k, constraint.get(k, nan))
    return b


class AugConfig(ctypes.Structure):
    _fields_ = [
        ("scale_min", ctypes.c_float), ("scale_max", ctypes.c_float),
        ("angle_min", ctypes.c_int), ("angle_max", ctypes.c_int),
        ("lighting_mean", ctypes.c_float), ("lighting_stddev", ctypes.c_float),
        ("hdist_min", ctypes.c_float), ("hdist_max", ctypes.c_float),
        ("contrast_min", ctypes.c_float), ("contrast_max", ctypes.c_float),
        ("brightness_min", ctypes.c_float), ("brightness_max", ctypes.c_float),
        ("saturation_min", ctypes.c_float), ("saturation_max", ctypes.c_float),
        ("hue_min", ctypes.c_int), ("hue_max", ctypes.c_int),
        ("flip_enable", ctypes.c_int), ("center", ctypes.c_int),
        ("crop_enable", ctypes.c_int), ("do_area_scale", ctypes.c_int),
        ("resize_short_size", ctypes.c_int), ("padding", ctypes.c_int),
        ("fixed_scaling_factor", ctypes.c_float),
        ("interp", ctypes.c_int),
        ("expand_probability", ctypes.c_float), ("expand_ratio_min", ctypes.c_float),
        ("expand_ratio_max", ctypes.c_float),
        ("n_samplers", ctypes.c_int), ("samplers", BatchSampler * 4),
    ]


class Params(ctypes.Structure):
    _fields_ = [
        ("crop_x", ctypes.c_int), ("crop_y", ctypes.c_int),
        ("crop_w", ctypes.c_int), ("crop_h", ctypes.c_int),
        ("resize_short_size", ctypes.c_int),
        ("out_w", ctypes.c_int), ("out_h", ctypes.c_int),
        ("angle", ctypes.c_int), ("flip", ctypes.c_int), ("padding", ctypes.c_int),
        ("pad_off_x", ctypes.c_int), ("pad_off_y", ctypes.c_int),
        ("n_lighting", ctypes.c_int), ("lighting", ctypes.c_float * 3),
        ("color_noise_std", ctypes.c_float),
        ("contrast", ctypes.c_float), ("brightness", ctypes.c_float),
        ("saturation", ctypes.c_float), ("hue", ctypes.c_int),
        ("interp", ctypes.c_int),
        ("expand_ratio", ctypes.c_float), ("expand_x", ctypes.c_int), ("expand_y", ctypes.c_int),
        ("expand_w", ctypes.c_int), ("expand_h", ctypes.c_int),
    ]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["lighting"] = list(self.lighting)
        return d


class LoadConfig(ctypes.Structure):
    _fields_ = [
        ("channels", ctypes.c_int), ("channel_major", ctypes.c_int),
        ("bgr_to_rgb", ctypes.c_int), ("out_dtype", ctypes.c_int),
        ("has_mean", ctypes.c_int),
        ("mean", ctypes.c_double * 3), ("stddev", ctypes.c_double * 3),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        L.orc_factory_create.restype = ctypes.c_void_p
        L.orc_factory_create.argtypes = [P(AugConfig)]
        L.orc_factory_destroy.argtypes = [ctypes.c_void_p]
        L.orc_make_params.argtypes = [ctypes.c_void_p, P(ctypes.c_uint32), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, P(Params)]
        L.orc_make_ssd_params.argtypes = [ctypes.c_void_p, P(ctypes.c_uint32), ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, P(ctypes.c_float), ctypes.c_int, P(Params)]
        L.orc_sample_patches.argtypes = [ctypes.c_void_p, ctypes.c_int, P(ctypes.c_uint32), P(ctypes.c_float),
                                         ctypes.c_int, P(ctypes.c_float), ctypes.c_int, P(ctypes.c_int)]
        L.orc_seed_slots.argtypes = [ctypes.c_uint32, ctypes.c_int, P(ctypes.c_uint32)]
        L.orc_transform_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, P(Params), ctypes.c_void_p]
        L.orc_load_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, P(LoadConfig),
                                     ctypes.c_void_p]
        L.orc_transform_mask.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         P(Params), ctypes.c_void_p]
        for fn in (L.orc_resize_linear, L.orc_resize_nearest):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.orc_resize_cv.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_lanczos4_coeffs.argtypes = [ctypes.c_float, P(ctypes.c_float)]
        L.orc_lanczos4_coeffs.restype = None
        L.orc_cbsjitter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                    ctypes.c_float, ctypes.c_float, ctypes.c_int]
        L.orc_lighting.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, P(ctypes.c_float),
                                   ctypes.c_int, ctypes.c_float]
        L.orc_u8_standardize_value.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.orc_standardize_value.restype = ctypes.c_float
        L.orc_standardize_value.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.orc_batch_augment.restype = ctypes.c_double
        L.orc_batch_augment.argtypes = [ctypes.c_int, P(ctypes.c_void_p), P(ctypes.c_int),
                                        P(ctypes.c_int), P(Params), P(LoadConfig), ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_int]
        L.orc_batch_image_mask.restype = ctypes.c_double
        L.orc_batch_image_mask.argtypes = [ctypes.c_int, P(ctypes.c_void_p), P(ctypes.c_void_p), P(ctypes.c_int),
                                           P(ctypes.c_int), P(Params), P(LoadConfig), ctypes.c_void_p,
                                           ctypes.c_size_t, P(LoadConfig), ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_int]
        L.orc_set_affinity.argtypes = [P(ctypes.c_int), ctypes.c_int]
        L.orc_set_affinity.restype = None
        L.orc_pool_cpus.argtypes = [ctypes.c_int, P(ctypes.c_int)]
        L.orc_pool_cpus.restype = None
        L.orc_rotate.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p]
        L.orc_transpose.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
        L.orc_unbiased_round.argtypes = [ctypes.c_float]
        L.orc_calculate_scale.restype = ctypes.c_float
        L.orc_calculate_scale.argtypes = [ctypes.c_int] * 4
        L.orc_cropbox_max_proportional.argtypes = [ctypes.c_float] * 4 + [P(ctypes.c_float)] * 2
        L.orc_jpeg_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t] + [P(ctypes.c_int)] * 3
        L.orc_jpeg_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.orc_jpeg_last_error.restype = ctypes.c_char_p
        L.orc_batch_decode_augment.restype = ctypes.c_double
        L.orc_batch_decode_augment.argtypes = [ctypes.c_int, P(ctypes.c_void_p), P(ctypes.c_size_t), P(Params),
                                               P(LoadConfig), ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        L.orc_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError("oracle: " + lib().orc_last_error().decode())


def aug_config(**kw):
    """AugConfig with aeon's param_factory defaults (augment_image.hpp:141-204)."""
    c = AugConfig(scale_min=1.0, scale_max=1.0, angle_min=0, angle_max=0,
                  lighting_mean=0.0, lighting_stddev=0.0, hdist_min=1.0, hdist_max=1.0,
                  contrast_min=1.0, contrast_max=1.0, brightness_min=1.0, brightness_max=1.0,
                  saturation_min=1.0, saturation_max=1.0, hue_min=0, hue_max=0,
                  flip_enable=0, center=1, crop_enable=1, do_area_scale=0,
                  resize_short_size=0, padding=0, fixed_scaling_factor=-1.0, interp=0,
                  expand_probability=0.0, expand_ratio_min=1.0, expand_ratio_max=1.0, n_samplers=0)
    for k, v in kw.items():
        if k == "samplers":
            c.n_samplers = len(v)
            for i, b in enumerate(v):
                c.samplers[i] = b
        else:
            setattr(c, k, v)
    return c


class Factory:
    def __init__(self, cfg):
        self._f = lib().orc_factory_create(ctypes.byref(cfg))

    def __del__(self):
        if getattr(self, "_f", None):
            lib().orc_factory_destroy(self._f)
            self._f = None

    def make_params(self, state, in_w, in_h, out_w, out_h):
        """state: 1-element np.uint32 array (the slot's engine state, updated in place)."""
        p = Params()
        st = ctypes.c_uint32(int(state[0]))
        _check(lib().orc_make_params(self._f, ctypes.byref(st), in_w, in_h, out_w, out_h,
                                     ctypes.byref(p)))
        state[0] = st.value
        return p


def make_ssd_params(factory, state, in_w, in_h, out_w, out_h, boxes=()):
    """param_factory::make_ssd_params; boxes: (xmin, ymin, xmax, ymax) per object."""
    p = Params()
    st = ctypes.c_uint32(int(state[0]))
    flat = (ctypes.c_float * max(1, 4 * len(boxes)))(*[v for b in boxes for v in b])
    _check(lib().orc_make_ssd_params(factory._f, ctypes.byref(st), in_w, in_h, out_w, out_h, flat, len(boxes),
                                     ctypes.byref(p)))
    state[0] = st.value
    return p


def sample_patches(factory, sampler, state, nboxes, cap=4096):
    """batch_sampler::sample_patches -> list of (xmin, ymin, xmax, ymax) normalized boxes."""
    st = ctypes.c_uint32(int(state[0]))
    flat = (ctypes.c_float * max(1, 4 * len(nboxes)))(*[v for b in nboxes for v in b])
    out = (ctypes.c_float * (4 * cap))()
    n = ctypes.c_int()
    _check(lib().orc_sample_patches(factory._f, sampler, ctypes.byref(st), flat, len(nboxes), out, cap,
                                    ctypes.byref(n)))
    state[0] = st.value
    return [tuple(out[4 * i:4 * i + 4]) for i in range(min(n.value, cap))]


def seed_slots(seed, n):
    out = np.zeros(n, np.uint32)
    lib().orc_seed_slots(seed, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    return out


def params(**kw):
    p = Params(interp=0, contrast=1.0, brightness=1.0, saturation=1.0)
    for k, v in kw.items():
        if k == "lighting":
            p.n_lighting = len(v)
            for i, x in enumerate(v):
                p.lighting[i] = x
        else:
            setattr(p, k, v)
    return p


def unbiased_round(x):
    return lib().orc_unbiased_round(x)


def calculate_scale(w, h, ow, oh):
    return lib().orc_calculate_scale(w, h, ow, oh)


def cropbox_max_proportional(in_w, in_h, out_w, out_h):
    rw, rh = ctypes.c_float(), ctypes.c_float()
    lib().orc_cropbox_max_proportional(in_w, in_h, out_w, out_h, ctypes.byref(rw), ctypes.byref(rh))
    return rw.value, rh.value


def jpeg_info(data):
    """(width, height, components) of a JPEG file's frame."""
    w, h, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if lib().orc_jpeg_info(bytes(data), len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n)) != 0:
        raise RuntimeError("oracle: " + lib().orc_jpeg_last_error().decode())
    return w.value, h.value, n.value


def jpeg_decode(data, channels=3):
    """cv::imdecode of a JPEG as aeon's extractor calls it: HWC BGR (channels 3) or gray (1)."""
    w, h, _ = jpeg_info(data)
    out = np.zeros((h, w, channels) if channels == 3 else (h, w), np.uint8)
    if lib().orc_jpeg_decode(bytes(data), len(data), channels, out.ctypes.data) != 0:
        raise RuntimeError("oracle: " + lib().orc_jpeg_last_error().decode())
    return out


def transform_image(src, p):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.zeros((p.out_h, p.out_w, cn), np.uint8)
    _check(lib().orc_transform_image(src.ctypes.data, w, h, cn, w * cn, ctypes.byref(p),
                                     out.ctypes.data))
    return out


DTYPES = {"uint8": (0, np.uint8), "float32": (1, np.float32), "int8": (2, np.int8), "int16": (3, np.int16),
          "uint16": (4, np.uint16), "int32": (5, np.int32), "float64": (6, np.float64)}
NP_OF = {code: t for code, t in DTYPES.values()}


def load_config(channels=3, channel_major=True, bgr_to_rgb=False, out_dtype="float32",
                mean=None, stddev=None):
    lc = LoadConfig(channels=channels, channel_major=int(channel_major), bgr_to_rgb=int(bgr_to_rgb),
                    out_dtype=DTYPES[out_dtype][0], has_mean=0)
    if mean is not None:
        lc.has_mean = 1
        for i in range(channels):
            lc.mean[i] = mean[i]
            lc.stddev[i] = stddev[i]
    return lc


def load_image(img, lc):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    dt = NP_OF[lc.out_dtype]
    shape = (lc.channels, h, w) if lc.channel_major else (h, w, lc.channels)
    out = np.zeros(shape, dt)
    _check(lib().orc_load_image(img.ctypes.data, w, h, ctypes.byref(lc), out.ctypes.data))
    return out


def transform_mask(src, p):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape[:2]
    out = np.zeros((p.out_h, p.out_w), np.uint8)
    _check(lib().orc_transform_mask(src.ctypes.data, w, h, w, ctypes.byref(p), out.ctypes.data))
    return out


def resize_linear(src, dw, dh):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.zeros((dh, dw, cn), np.uint8)
    _check(lib().orc_resize_linear(src.ctypes.data, w, h, w * cn, cn, out.ctypes.data, dw, dh))
    return out


INTERP = {"LINEAR": 0, "NEAREST": 1, "CUBIC": 2, "AREA": 3, "LANCZOS4": 4}


def resize(src, dw, dh, interp):
    """cv::resize (OpenCV 2.4.9) of HWC uint8 with interpolation code or name (INTERP)."""
    code = INTERP[interp.upper()] if isinstance(interp, str) else int(interp)
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.zeros((dh, dw) + (() if src.ndim == 2 else (cn,)), np.uint8)
    _check(lib().orc_resize_cv(src.ctypes.data, w, h, w * cn, cn, out.ctypes.data, dw, dh, code))
    return out


def lanczos4_coeffs(x):
    out = (ctypes.c_float * 8)()
    lib().orc_lanczos4_coeffs(x, out)
    return np.array(out[:], np.float32)


def resize_nearest(src, dw, dh):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.zeros((dh, dw, cn), np.uint8)
    _check(lib().orc_resize_nearest(src.ctypes.data, w, h, w * cn, cn, out.ctypes.data, dw, dh))
    return out


def cbsjitter(img, contrast=1.0, brightness=1.0, saturation=1.0, hue=0):
    img = np.ascontiguousarray(img, dtype=np.uint8).copy()
    h, w = img.shape[:2]
    lib().orc_cbsjitter(img.ctypes.data, w, h, contrast, brightness, saturation, hue)
    return img


def lighting(img, alphas, sigma):
    img = np.ascontiguousarray(img, dtype=np.uint8).copy()
    h, w = img.shape[:2]
    a = (ctypes.c_float * 3)(*alphas)
    lib().orc_lighting(img.ctypes.data, w, h, a, len(alphas), sigma)
    return img


def augment_record(src, p, lc):
    """transform_single_image + loader::load for one record."""
    return load_image(transform_image(src, p), lc)


def u8_standardize(x, mean, stddev):
    """uint8 result of standardizing a CV_8U canvas value x (fixed_aspect_ratio loader)."""
    return lib().orc_u8_standardize_value(int(x), mean, stddev)


def set_affinity(cpus):
    """Pin the baseline pool like aeon's thread_pool: worker t on cpus[t % len(cpus)]; [] = unpinned."""
    arr = (ctypes.c_int * max(1, len(cpus)))(*cpus)
    lib().orc_set_affinity(arr, len(cpus))


def pool_cpus(threads):
    """The single CPU each of `threads` baseline-pool workers is pinned to (-1: not pinned to one)."""
    out = (ctypes.c_int * max(1, threads))()
    lib().orc_pool_cpus(threads, out)
    return list(out[:threads])


def batch_augment(srcs, params_list, lc, item_shape, threads):
    """CPU-baseline batch on `threads` pool workers; returns (outputs, seconds)."""
    n = len(srcs)
    srcs = [np.ascontiguousarray(s, dtype=np.uint8) for s in srcs]
    ptrs = (ctypes.c_void_p * n)(*[s.ctypes.data for s in srcs])
    ws = (ctypes.c_int * n)(*[s.shape[1] for s in srcs])
    hs = (ctypes.c_int * n)(*[s.shape[0] for s in srcs])
    ps = (Params * n)(*params_list)
    dt = np.uint8 if lc.out_dtype == 0 else np.float32
    out = np.zeros((n,) + tuple(item_shape), dt)
    item_bytes = out[0].nbytes
    secs = lib().orc_batch_augment(n, ptrs, ws, hs, ps, ctypes.byref(lc), out.ctypes.data,
                                   item_bytes, threads)
    if secs < 0:
        raise RuntimeError("oracle: " + lib().orc_last_error().decode())
    return out, secs


def batch_image_mask(srcs, masks, params_list, lc, item_shape, mlc, mask_shape, threads):
    """CPU-baseline batch of image + pixelmask pairs sharing params; returns (img, mask, seconds)."""
    n = len(srcs)
    srcs = [np.ascontiguousarray(s, dtype=np.uint8) for s in srcs]
    masks = [np.ascontiguousarray(m, dtype=np.uint8) for m in masks]
    ptrs = (ctypes.c_void_p * n)(*[s.ctypes.data for s in srcs])
    mptrs = (ctypes.c_void_p * n)(*[m.ctypes.data for m in masks])
    ws = (ctypes.c_int * n)(*[s.shape[1] for s in srcs])
    hs = (ctypes.c_int * n)(*[s.shape[0] for s in srcs])
    ps = (Params * n)(*params_list)
    out = np.zeros((n,) + tuple(item_shape), np.uint8 if lc.out_dtype == 0 else np.float32)
    mout = np.zeros((n,) + tuple(mask_shape), np.uint8 if mlc.out_dtype == 0 else np.float32)
    secs = lib().orc_batch_image_mask(n, ptrs, mptrs, ws, hs, ps, ctypes.byref(lc), out.ctypes.data, out[0].nbytes,
                                      ctypes.byref(mlc), mout.ctypes.data, mout[0].nbytes, threads)
    if secs < 0:
        raise RuntimeError("oracle: " + lib().orc_last_error().decode())
    return out, mout, secs


def batch_decode_augment(files, params_list, lc, item_shape, threads):
    """aeon's CPU path (JPEG decode + transform + load) over encoded files; returns (out, seconds)."""
    n = len(files)
    bufs = [bytes(f) for f in files]
    ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in bufs])
    sizes = (ctypes.c_size_t * n)(*[len(b) for b in bufs])
    ps = (Params * n)(*params_list)
    out = np.zeros((n,) + tuple(item_shape), np.uint8 if lc.out_dtype == 0 else np.float32)
    secs = lib().orc_batch_decode_augment(n, ptrs, sizes, ps, ctypes.byref(lc), out.ctypes.data, out[0].nbytes, threads)
    if secs < 0:
        raise RuntimeError("oracle: " + lib().orc_last_error().decode())
    return out, secs


def transpose(src, rows, cols, element_size):
    """transpose_buf: bytes of a rows x cols matrix of element_size-byte elements, transposed."""
    src = np.ascontiguousarray(src).view(np.uint8).reshape(-1)
    if src.size != rows * cols * element_size:
        raise ValueError("size mismatch")
    out = np.empty_like(src)
    _check(lib().orc_transpose(out.ctypes.data, src.ctypes.data, ctypes.c_int64(rows), ctypes.c_int64(cols),
                               element_size))
    return out


def rotate(src, angle, interpolate=True):
    """image::rotate: warpAffine about (cols/2, rows/2), linear or nearest, zero border."""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape[:2]
    cn = 1 if src.ndim == 2 else src.shape[2]
    out = np.empty_like(src)
    _check(lib().orc_rotate(src.ctypes.data, w, h, cn, w * cn, angle, int(interpolate), out.ctypes.data))
    return out
