"""aeon_amd -- MI355X (gfx950) image-augmentation stage for NervanaSystems/aeon.

Python binding of the C ABI in include/aeon_hip.h (libaeon_hip.so, built in-tree).
The pixel path runs only in the HIP kernels of that library: there is no CPU fallback, and
importing this package fails loudly when the library is missing.  PyTorch is used only as
plumbing (device memory and streams) by callers; the binding itself takes raw pointers.
"""
import ctypes
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# AEON_HIP_LIB: a kernel tuning variant built by tools/build_variants.sh (development only)
LIB_PATH = os.environ.get("AEON_HIP_LIB") or os.path.join(HERE, "libaeon_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "aeon_hip.h")

AEON_HIP_OK = 0
AEON_HIP_EINVAL = -1
AEON_HIP_ERUNTIME = -2
AEON_HIP_EUNSUPPORTED = -3
AEON_HIP_EDEVICE = -4

DTYPE_U8 = 0
DTYPE_F32 = 1
# output dtype name -> (AEON_DTYPE_* code, numpy type); aeon output_type uint32_t maps to int32 storage
DTYPES = {"uint8": (0, np.uint8), "float32": (1, np.float32), "int8": (2, np.int8), "int16": (3, np.int16),
          "uint16": (4, np.uint16), "int32": (5, np.int32), "float64": (6, np.float64)}
NP_DTYPE = {code: t for code, t in DTYPES.values()}
INTERP_LINEAR = 0
INTERP_NEAREST = 1
INTERP_CUBIC = 2
INTERP_AREA = 3
INTERP_LANCZOS4 = 4


class ImgDesc(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("stride", ctypes.c_int32), ("channels", ctypes.c_int32), ("elem_bytes", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class AugParams(ctypes.Structure):
    """POD mirror of augment::image::params (aeon src/augment_image.hpp:99-119)."""
    _fields_ = [
        ("crop_x", ctypes.c_int32), ("crop_y", ctypes.c_int32),
        ("crop_w", ctypes.c_int32), ("crop_h", ctypes.c_int32),
        ("resize_short_size", ctypes.c_int32),
        ("out_w", ctypes.c_int32), ("out_h", ctypes.c_int32),
        ("angle", ctypes.c_int32), ("flip", ctypes.c_int32),
        ("padding", ctypes.c_int32), ("pad_off_x", ctypes.c_int32), ("pad_off_y", ctypes.c_int32),
        ("n_lighting", ctypes.c_int32), ("lighting", ctypes.c_float * 3),
        ("color_noise_std", ctypes.c_float),
        ("contrast", ctypes.c_float), ("brightness", ctypes.c_float),
        ("saturation", ctypes.c_float), ("hue", ctypes.c_int32),
        ("interp", ctypes.c_int32),
        ("expand_ratio", ctypes.c_float), ("expand_x", ctypes.c_int32), ("expand_y", ctypes.c_int32),
        ("expand_w", ctypes.c_int32), ("expand_h", ctypes.c_int32),
    ]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["lighting"] = list(self.lighting)
        return d


class OutDesc(ctypes.Structure):
    """image::loader configuration + batch item stride (aeon src/etl_image.cpp:204-244)."""
    _fields_ = [("dtype", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("channel_major", ctypes.c_int32), ("bgr_to_rgb", ctypes.c_int32),
                ("has_mean", ctypes.c_int32), ("fixed_aspect_ratio", ctypes.c_int32),
                ("mean", ctypes.c_double * 3), ("stddev", ctypes.c_double * 3),
                ("item_stride", ctypes.c_uint64), ("canvas_w", ctypes.c_int32), ("canvas_h", ctypes.c_int32)]


class RecordElem(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("stride", ctypes.c_int32)]


class EncodedElem(ctypes.Structure):
    """aeon_encoded_elem: an encoded JPEG file (width 0) or decoded HWC uint8 pixels."""
    _fields_ = [("data", ctypes.c_void_p), ("size", ctypes.c_size_t), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("channels", ctypes.c_int32), ("stride", ctypes.c_int32)]


class EncodedRecords:
    """Records marshalled once (Decoder.encoded): their aeon_encoded_elem array and the Python objects
    whose memory it points at."""

    def __init__(self, n, elems, keep):
        self.n, self.elems, self.keep = n, elems, keep

    def __len__(self):
        return self.n


class AeonHipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"aeon_hip error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load libaeon_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`"
                              " (the HIP extension is required; there is no CPU fallback)")
        # One HIP runtime per process: PyTorch ships its own libamdhip64 (SONAME libamdhip64.so.7,
        # loaded by file name).  Loaded first, it also satisfies this library's dependency, so
        # torch streams/events and this library's launches share one runtime.  Loaded after this
        # library, it would bring a second runtime whose queues are not ordered with ours.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        vp = ctypes.c_void_p
        L.aeon_hip_ctx_create.argtypes = [ctypes.c_int, P(vp)]
        L.aeon_hip_ctx_destroy.argtypes = [vp]
        for fn in (L.aeon_hip_augment_batch, L.aeon_hip_mask_batch, L.aeon_hip_depthmap_batch):
            fn.argtypes = [vp, ctypes.c_int, P(ImgDesc), vp, P(AugParams), P(OutDesc), vp, vp]
        if hasattr(L, "aeon_hip_augment_pair_batch"):  # absent only in older tuning-variant builds
            L.aeon_hip_augment_pair_batch.argtypes = [vp, ctypes.c_int, P(ImgDesc), vp, P(ImgDesc), vp, P(AugParams),
                                                      P(OutDesc), vp, P(OutDesc), vp, vp]
        L.aeon_hip_synchronize.argtypes = [vp, vp]
        if hasattr(L, "aeon_hip_transpose_batch"):  # absent only in older tuning-variant builds
            L.aeon_hip_transpose_batch.argtypes = [vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, vp]
        L.aeon_hip_set_timing.argtypes = [vp, ctypes.c_int]
        L.aeon_hip_kernel_times.argtypes = [vp, ctypes.c_int, P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_long)]
        L.aeon_param_factory_create.argtypes = [ctypes.c_char_p, P(vp)]
        L.aeon_param_factory_destroy.argtypes = [vp]
        L.aeon_make_params.argtypes = [vp, P(ctypes.c_uint32), ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int, P(AugParams)]
        L.aeon_make_ssd_params.argtypes = [vp, P(ctypes.c_uint32), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, P(ctypes.c_float), ctypes.c_int, P(AugParams)]
        L.aeon_batch_sample_patches.argtypes = [vp, ctypes.c_int, P(ctypes.c_uint32), P(ctypes.c_float),
                                                ctypes.c_int, P(ctypes.c_float), ctypes.c_int, P(ctypes.c_int)]
        L.aeon_seed_slots.argtypes = [ctypes.c_uint32, ctypes.c_int, P(ctypes.c_uint32)]
        L.aeon_unbiased_round.argtypes = [ctypes.c_float, P(ctypes.c_int64)]
        L.aeon_calculate_scale.argtypes = [ctypes.c_int] * 4 + [P(ctypes.c_float)]
        L.aeon_cropbox_max_proportional.argtypes = [ctypes.c_float] * 4 + [P(ctypes.c_float)] * 2
        L.aeon_jpeg_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t] + [P(ctypes.c_int)] * 3
        L.aeon_jpeg_entropy_decode.argtypes = ([ctypes.c_char_p, ctypes.c_size_t] + [P(ctypes.c_int)] * 3 +
                                               [P(ctypes.c_int64)] * 2 + [P(ctypes.c_uint64)])
        L.aeon_jpeg_host_stage.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P(ctypes.c_int), P(ctypes.c_int64)]
        L.aeon_png_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t] + [P(ctypes.c_int)] * 4
        L.aeon_decode_png.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, vp, ctypes.c_size_t,
                                      P(ctypes.c_int)]
        L.aeon_hip_decode_jpeg_batch.argtypes = [vp, ctypes.c_int, P(vp), P(ctypes.c_size_t), P(ImgDesc), vp, vp]
        L.aeon_hip_stager_create.argtypes = [vp, ctypes.c_int, P(OutDesc), ctypes.c_int, P(vp)]
        L.aeon_hip_stager_destroy.argtypes = [vp]
        L.aeon_hip_stager_stage.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, P(AugParams)]
        L.aeon_hip_stager_flush.argtypes = [vp, vp]
        L.aeon_hip_stager_launch.argtypes = [vp, vp]
        L.aeon_hip_stager_wait.argtypes = [vp, vp]
        L.aeon_hip_release_stream.argtypes = [vp, vp]
        L.aeon_hip_stager_last_error.restype = ctypes.c_char_p
        L.aeon_hip_host_alloc.argtypes = [ctypes.c_size_t, P(vp)]
        L.aeon_hip_host_free.argtypes = [vp]
        L.aeon_decoder_create.argtypes = [ctypes.c_char_p, ctypes.c_int, P(vp)]
        L.aeon_decoder_destroy.argtypes = [vp]
        L.aeon_decoder_output_count.argtypes = [vp, P(ctypes.c_int)]
        L.aeon_decoder_output_info.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                               P(ctypes.c_int64), P(ctypes.c_int), P(ctypes.c_size_t),
                                               P(ctypes.c_int)]
        L.aeon_decoder_decode.argtypes = [vp, ctypes.c_int, P(RecordElem), P(vp), ctypes.c_int, vp]
        L.aeon_decoder_decode_encoded.argtypes = [vp, ctypes.c_int, P(EncodedElem), P(vp), ctypes.c_int, vp]
        L.aeon_decoder_draw_params.argtypes = [vp, ctypes.c_int, P(RecordElem), P(AugParams), ctypes.c_int]
        L.aeon_decoder_submit.argtypes = [vp, ctypes.c_int, P(EncodedElem), P(vp), ctypes.c_int]
        L.aeon_decoder_wait.argtypes = [vp]
        L.aeon_decoder_last_error.restype = ctypes.c_char_p
        L.aeon_thread_affinity_map.argtypes = [ctypes.c_char_p, P(ctypes.c_int), ctypes.c_int, P(ctypes.c_int)]
        L.aeon_decoder_pool_size.argtypes = [vp, P(ctypes.c_int)]
        L.aeon_decoder_pool_cpus.argtypes = [vp, ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int), ctypes.c_int,
                                             P(ctypes.c_int)]
        L.aeon_manifest_node_slice.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               P(ctypes.c_int64), P(ctypes.c_int64)]
        L.aeon_hip_last_error.restype = ctypes.c_char_p
        L.aeon_hip_version.restype = ctypes.c_char_p
        L.aeon_hip_debug_uncached_blocks.argtypes = [P(ctypes.c_uint64), ctypes.c_int, P(ctypes.c_int)]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise AeonHipError(rc, lib().aeon_hip_last_error().decode())
    return rc


def uncached_blocks():
    """[(lo, hi)] device address ranges of every uncached job-table block of this process (diagnostics:
    aeon_hip_debug_uncached_blocks)."""
    n = ctypes.c_int()
    _check(lib().aeon_hip_debug_uncached_blocks(None, 0, ctypes.byref(n)))
    buf = (ctypes.c_uint64 * (2 * max(n.value, 1)))()
    _check(lib().aeon_hip_debug_uncached_blocks(buf, n.value, ctypes.byref(n)))
    return [(buf[2 * i], buf[2 * i + 1]) for i in range(n.value)]


def exported_symbols():
    """Function names declared in include/aeon_hip.h."""
    import re
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(aeon_\w+)\s*\(", text, re.M)))


# ---- parameters (host) -------------------------------------------------------------------------
class ParamFactory:
    """augment::image::param_factory (aeon src/augment_image.cpp:28-230)."""

    def __init__(self, aug_config):
        text = aug_config if isinstance(aug_config, str) else json.dumps(aug_config)
        h = ctypes.c_void_p()
        _check(lib().aeon_param_factory_create(text.encode(), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.aeon_param_factory_destroy(self._h)
            self._h = None

    def make_params(self, state, in_w, in_h, out_w, out_h):
        """state: np.uint32 array of one element (minstd_rand0 state word, updated in place)."""
        p = AugParams()
        st = ctypes.c_uint32(int(state[0]))
        _check(lib().aeon_make_params(self._h, ctypes.byref(st), in_w, in_h, out_w, out_h, ctypes.byref(p)))
        state[0] = st.value
        return p

    def sample_patches(self, sampler, state, nboxes, cap=4096):
        """batch_sampler::sample_patches of batch_samplers[sampler] (aeon src/augment_image.cpp:567-586)
        over normalized boxes; returns the sampled normalized boxes."""
        st = ctypes.c_uint32(int(state[0]))
        flat = (ctypes.c_float * max(1, 4 * len(nboxes)))(*[float(v) for b in nboxes for v in b])
        out = (ctypes.c_float * (4 * cap))()
        n = ctypes.c_int()
        _check(lib().aeon_batch_sample_patches(self._h, sampler, ctypes.byref(st), flat, len(nboxes), out, cap,
                                               ctypes.byref(n)))
        state[0] = st.value
        return [tuple(out[4 * i:4 * i + 4]) for i in range(min(n.value, cap))]

    def make_ssd_params(self, state, in_w, in_h, out_w, out_h, boxes=()):
        """param_factory::make_ssd_params (aeon src/augment_image.cpp:232-310); boxes are
        boundingbox::box pixel coordinates (xmin, ymin, xmax, ymax), xmax/ymax inclusive."""
        p = AugParams()
        st = ctypes.c_uint32(int(state[0]))
        flat = (ctypes.c_float * max(1, 4 * len(boxes)))(*[float(v) for b in boxes for v in b])
        _check(lib().aeon_make_ssd_params(self._h, ctypes.byref(st), in_w, in_h, out_w, out_h, flat, len(boxes),
                                          ctypes.byref(p)))
        state[0] = st.value
        return p


def seed_slots(seed, n):
    """batch_decoder deterministic-mode engine states (aeon src/batch_decoder.cpp:47-54)."""
    out = np.zeros(n, np.uint32)
    _check(lib().aeon_seed_slots(seed, n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))))
    return out


def jpeg_info(data):
    """(width, height, components) of a JPEG file (aeon_jpeg_info)."""
    w, h, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().aeon_jpeg_info(bytes(data), len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n)))
    return w.value, h.value, n.value


def jpeg_entropy_decode(data):
    """Host-only Huffman decode of a JPEG file (aeon_jpeg_entropy_decode): (width, height,
    components, blocks, non-zero values, FNV-1a hash of the sparse coefficient stream)."""
    w, h, n = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    nb, nv, hv = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_uint64()
    _check(lib().aeon_jpeg_entropy_decode(bytes(data), len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(n),
                                          ctypes.byref(nb), ctypes.byref(nv), ctypes.byref(hv)))
    return w.value, h.value, n.value, nb.value, nv.value, hv.value


def jpeg_host_stage(data):
    """The JPEG batch decode's host work for one file (aeon_jpeg_host_stage): (GPU entropy decoding?,
    bytes staged for the H2D)."""
    g, nb = ctypes.c_int(), ctypes.c_int64()
    _check(lib().aeon_jpeg_host_stage(bytes(data), len(data), ctypes.byref(g), ctypes.byref(nb)))
    return bool(g.value), nb.value


PNG_BGR8, PNG_GRAY8, PNG_ANYDEPTH = 0, 1, 2


def png_info(data):
    """(width, height, bit depth, PNG colour type) of a PNG file (aeon_png_info)."""
    w, h, d, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(lib().aeon_png_info(bytes(data), len(data), ctypes.byref(w), ctypes.byref(h), ctypes.byref(d),
                               ctypes.byref(c)))
    return w.value, h.value, d.value, c.value


def decode_png(data, mode=PNG_BGR8):
    """cv::imdecode of a PNG file as aeon's extractors ask for it (aeon_decode_png): HxWx3 uint8 BGR
    (PNG_BGR8), HxW uint8 (PNG_GRAY8), or HxW uint8 / uint16 at the file's depth (PNG_ANYDEPTH)."""
    w, h, d, c = png_info(data)
    wide = mode == PNG_ANYDEPTH and d == 16 and c != 3
    cn = 3 if mode == PNG_BGR8 else 1
    out = np.zeros((h, w, cn) if cn == 3 else (h, w), np.uint16 if wide else np.uint8)
    eb = ctypes.c_int()
    _check(lib().aeon_decode_png(bytes(data), len(data), mode, out.ctypes.data, out.strides[0], ctypes.byref(eb)))
    return out


def unbiased_round(x):
    """nervana::unbiased_round (aeon src/util.cpp:212-239)."""
    r = ctypes.c_int64()
    _check(lib().aeon_unbiased_round(x, ctypes.byref(r)))
    return r.value


def calculate_scale(w, h, out_w, out_h):
    """image::calculate_scale (aeon src/image.cpp:214-224)."""
    s = ctypes.c_float()
    _check(lib().aeon_calculate_scale(w, h, out_w, out_h, ctypes.byref(s)))
    return s.value


def cropbox_max_proportional(in_w, in_h, out_w, out_h):
    """image::cropbox_max_proportional (aeon src/image.cpp:226-237) -> (width, height)."""
    rw, rh = ctypes.c_float(), ctypes.c_float()
    _check(lib().aeon_cropbox_max_proportional(in_w, in_h, out_w, out_h, ctypes.byref(rw), ctypes.byref(rh)))
    return rw.value, rh.value


def aug_params(**kw):
    p = AugParams(contrast=1.0, brightness=1.0, saturation=1.0, interp=INTERP_LINEAR)
    for k, v in kw.items():
        if k == "lighting":
            p.n_lighting = len(v)
            for i, x in enumerate(v):
                p.lighting[i] = x
        else:
            setattr(p, k, v)
    return p


def out_desc(channels=3, channel_major=True, bgr_to_rgb=False, dtype="float32", mean=None,
             stddev=None, item_stride=0, fixed_aspect_ratio=False, canvas=(0, 0)):
    o = OutDesc(dtype=DTYPES[dtype][0], channels=channels,
                channel_major=int(channel_major), bgr_to_rgb=int(bgr_to_rgb), has_mean=0,
                item_stride=item_stride, fixed_aspect_ratio=int(fixed_aspect_ratio),
                canvas_w=canvas[0], canvas_h=canvas[1])
    if mean is not None:
        o.has_mean = 1
        for i in range(channels):
            o.mean[i] = mean[i]
            o.stddev[i] = stddev[i]
    return o


# ---- device stage --------------------------------------------------------------------------------
class JpegFiles:
    """Encoded files marshalled once for aeon_hip_decode_jpeg_batch (the pointer and size arrays; the
    bytes objects are kept alive here)."""

    def __init__(self, files):
        self.bufs = [bytes(f) for f in files]
        n = len(self.bufs)
        self.ptrs = (ctypes.c_void_p * n)(*[ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) for b in self.bufs])
        self.sizes = (ctypes.c_size_t * n)(*[len(b) for b in self.bufs])

    def __len__(self):
        return len(self.bufs)


class Context:
    """One per GPU (aeon_hip_ctx)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        _check(lib().aeon_hip_ctx_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            _check(lib().aeon_hip_ctx_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _batch(self, fn, descs, src_ptr, params, out, out_ptr, stream):
        n = len(descs)
        # prebuilt ctypes arrays pass straight through (the C++ host fills these in place)
        d = descs if isinstance(descs, ctypes.Array) else (ImgDesc * n)(*descs)
        p = params if isinstance(params, ctypes.Array) else (AugParams * n)(*params)
        if len(p) < n:
            raise ValueError(f"{len(p)} params for {n} records")
        _check(fn(self._h, n, d, ctypes.c_void_p(src_ptr), p, ctypes.byref(out),
                  ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream or 0)))

    def augment_batch(self, descs, src_ptr, params, out, out_ptr, stream=0):
        """transform_single_image + loader::load for len(descs) records (async on stream)."""
        self._batch(lib().aeon_hip_augment_batch, descs, src_ptr, params, out, out_ptr, stream)

    def mask_batch(self, descs, src_ptr, params, out, out_ptr, stream=0):
        """pixel_mask transform + load for len(descs) records (async on stream)."""
        self._batch(lib().aeon_hip_mask_batch, descs, src_ptr, params, out, out_ptr, stream)

    def pair_batch(self, descs, src_ptr, mask_descs, mask_src_ptr, params, out, out_ptr, mask_out, mask_out_ptr,
                   stream=0):
        """provider::image + provider::pixelmask of the same records, one params set per record
        (aeon_hip_augment_pair_batch: for 8-bit unrotated masks into uint8 items one job table and two
        launches -- the image tiles, then the masks' gather; AEON_HIP_FUSE_MASKS=1: one launch)."""
        n = len(descs)
        d = descs if isinstance(descs, ctypes.Array) else (ImgDesc * n)(*descs)
        md = mask_descs if isinstance(mask_descs, ctypes.Array) else (ImgDesc * n)(*mask_descs)
        p = params if isinstance(params, ctypes.Array) else (AugParams * n)(*params)
        if len(md) < n or len(p) < n:
            raise ValueError(f"{len(md)} masks / {len(p)} params for {n} records")
        _check(lib().aeon_hip_augment_pair_batch(self._h, n, d, ctypes.c_void_p(src_ptr), md, ctypes.c_void_p(mask_src_ptr),
                                                 p, ctypes.byref(out), ctypes.c_void_p(out_ptr), ctypes.byref(mask_out),
                                                 ctypes.c_void_p(mask_out_ptr), ctypes.c_void_p(stream or 0)))

    def depthmap_batch(self, descs, src_ptr, params, out, out_ptr, stream=0):
        """depthmap transform + load (aeon src/etl_depthmap.cpp) for len(descs) records."""
        self._batch(lib().aeon_hip_depthmap_batch, descs, src_ptr, params, out, out_ptr, stream)

    def decode_jpeg_batch(self, files, descs, dst_ptr, stream=0):
        """image::extractor::extract of JPEG files into device memory (aeon_hip_decode_jpeg_batch):
        files = list of bytes (or a JpegFiles, marshalled once), descs[i] = where record i goes (HWC,
        channels 3 = BGR / 1 = gray)."""
        jf = files if isinstance(files, JpegFiles) else JpegFiles(files)
        n, ptrs, sizes = len(jf), jf.ptrs, jf.sizes
        d = descs if isinstance(descs, ctypes.Array) else (ImgDesc * n)(*descs)
        _check(lib().aeon_hip_decode_jpeg_batch(self._h, n, ptrs, sizes, d, ctypes.c_void_p(dst_ptr),
                                                ctypes.c_void_p(stream or 0)))

    def set_timing(self, every=1):
        """Time the launches of one call in `every` (0 = off) with HIP events on their stream."""
        _check(lib().aeon_hip_set_timing(self._h, int(every)))

    def kernel_times(self):
        """{'augment'|'stats'|'pre'|'jpeg': (total_ms, total_algorithmic_bytes, launches)}"""
        ms, by, ct = (ctypes.c_double * 4)(), (ctypes.c_double * 4)(), (ctypes.c_long * 4)()
        _check(lib().aeon_hip_kernel_times(self._h, 4, ms, by, ct))
        return {k: (ms[i], by[i], ct[i]) for i, k in enumerate(("augment", "stats", "pre", "jpeg"))}

    def synchronize(self, stream=0):
        _check(lib().aeon_hip_synchronize(self._h, ctypes.c_void_p(stream or 0)))

    def release_stream(self, stream):
        """The caller is about to destroy `stream` (aeon_hip_release_stream)."""
        _check(lib().aeon_hip_release_stream(self._h, ctypes.c_void_p(stream or 0)))

    def transpose_batch(self, src_ptr, dst_ptr, rows, cols, element_size, stream=0):
        """batch_major=false layout: dst[c*rows + r] = src[r*cols + c] (async on stream)."""
        _check(lib().aeon_hip_transpose_batch(self._h, ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr),
                                              rows, cols, element_size, ctypes.c_void_p(stream or 0)))


STAGER_IMAGE, STAGER_MASK, STAGER_DEVICE_OUT = 0, 1, 0x100


def _check_stager(rc):
    if rc != 0:
        raise AeonHipError(rc, lib().aeon_hip_stager_last_error().decode())
    return rc


class Stager:
    """aeon_hip_stager: what the aeon-side provider::image / ::pixelmask hold.
    stage() from provide() on any pool thread (the ctypes call releases the GIL); launch() from
    post_process() once per batch (the first launch of a window launches the whole window and
    returns), wait() from the consumer before it reads a batch (wait_buffer(): by buffer alone, as
    batch_iterator_fbm::filler calls it); flush() = launch + wait."""

    def __init__(self, ctx, out, batch_size, kind=STAGER_IMAGE):
        h = ctypes.c_void_p()
        self._out = out
        _check_stager(lib().aeon_hip_stager_create(ctx._h, kind, ctypes.byref(out), batch_size, ctypes.byref(h)))
        self._h = h

    def stage(self, batch_out, idx, pixels, params):
        """pixels: HxWxC or HxW uint8 / uint16 array (host)."""
        a = np.ascontiguousarray(pixels)
        h, w = a.shape[:2]
        cn = 1 if a.ndim == 2 else a.shape[2]
        _check_stager(lib().aeon_hip_stager_stage(self._h, ctypes.c_void_p(batch_out), idx, a.ctypes.data, w, h,
                                                   a.strides[0], cn, a.itemsize, ctypes.byref(params)))

    def flush(self, batch_out):
        _check_stager(lib().aeon_hip_stager_flush(self._h, ctypes.c_void_p(batch_out)))

    def launch(self, batch_out):
        _check_stager(lib().aeon_hip_stager_launch(self._h, ctypes.c_void_p(batch_out)))

    def wait(self, batch_out):
        _check_stager(lib().aeon_hip_stager_wait(self._h, ctypes.c_void_p(batch_out)))

    @staticmethod
    def wait_buffer(batch_out):
        """aeon_hip_stager_wait(NULL, batch_out): whichever stager launched the buffer, if any."""
        _check_stager(lib().aeon_hip_stager_wait(None, ctypes.c_void_p(batch_out)))

    def close(self):
        if getattr(self, "_h", None):
            lib().aeon_hip_stager_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_images(images, align=16):
    """Concatenate HWC uint8 images into one byte arena; returns (arena, [ImgDesc])."""
    descs, chunks, off = [], [], 0
    for im in images:
        im = np.ascontiguousarray(im, dtype=np.uint8)
        h, w = im.shape[:2]
        cn = 1 if im.ndim == 2 else im.shape[2]
        descs.append(ImgDesc(offset=off, width=w, height=h, stride=w * cn, channels=cn))
        b = im.reshape(-1)
        pad = (-b.size) % align
        chunks.append(b)
        if pad:
            chunks.append(np.zeros(pad, np.uint8))
        off += b.size + pad
    arena = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
    return arena, descs


def synthetic_image(index, w, h, cn=3, seed=0x5EED):
    """Counter-based synthetic HWC uint8 image: byte = splitmix64(seed^(img<<32)^idx)&0xFF."""
    idx = np.arange(w * h * cn, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) ^ (np.uint64(index) << np.uint64(32)) ^ idx) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFF)).astype(np.uint8).reshape(h, w, cn) if cn > 1 else \
        (z & np.uint64(0xFF)).astype(np.uint8).reshape(h, w)


# ---- decode stage (provider_factory + batch_decoder, host C++) -----------------------------------
def _check_host(rc):
    if rc != 0:
        raise AeonHipError(rc, lib().aeon_decoder_last_error().decode())
    return rc


class Decoder:
    """aeon batch_decoder over provider_factory::create(config): decode windows of decoded
    records (one HWC uint8 array per ETL element) into the provider output buffers."""

    def __init__(self, config, device=0):
        text = config if isinstance(config, str) else json.dumps(config)
        h = ctypes.c_void_p()
        _check_host(lib().aeon_decoder_create(text.encode(), device, ctypes.byref(h)))
        self._h = h
        n = ctypes.c_int()
        _check_host(lib().aeon_decoder_output_count(self._h, ctypes.byref(n)))
        self.outputs = []
        for i in range(n.value):
            name = ctypes.create_string_buffer(256)
            shape = (ctypes.c_int64 * 8)()
            nd, ib, dt = ctypes.c_int(), ctypes.c_size_t(), ctypes.c_int()
            _check_host(lib().aeon_decoder_output_info(self._h, i, name, 256, shape, ctypes.byref(nd),
                                                       ctypes.byref(ib), ctypes.byref(dt)))
            self.outputs.append({"name": name.value.decode(), "shape": tuple(shape[:nd.value]),
                                 "item_bytes": ib.value,
                                 "dtype": NP_DTYPE.get(dt.value)})

    def close(self):
        if getattr(self, "_h", None):
            lib().aeon_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encoded(self, records):
        """The records marshalled once into their aeon_encoded_elem array (EncodedRecords), for windows
        submitted again and again: aeon's host hands the decoder plain pointers, so a benchmark that
        rebuilds ctypes structures per record per window (~2-5 us each) would time Python instead."""
        elems, keep = self._encoded(records)
        return EncodedRecords(len(records), elems, keep)

    def _encoded(self, records):
        """aeon_encoded_elem array for records whose elements are JPEG bytes or HWC uint8 arrays."""
        if isinstance(records, EncodedRecords):
            return records.elems, records.keep
        n, ne = len(records), len(self.outputs)
        keep = []
        elems = (EncodedElem * (n * ne))()
        for i, rec in enumerate(records):
            for k in range(ne):
                x = rec[k]
                if isinstance(x, (bytes, bytearray, memoryview)):
                    b = bytes(x)
                    keep.append(b)
                    elems[i * ne + k] = EncodedElem(ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p), len(b), 0, 0, 0, 0)
                else:
                    a = np.ascontiguousarray(x, dtype=np.uint8)
                    keep.append(a)
                    h, w = a.shape[:2]
                    cn = 1 if a.ndim == 2 else a.shape[2]
                    elems[i * ne + k] = EncodedElem(a.ctypes.data, a.nbytes, w, h, cn, w * cn)
        return elems, keep

    def decode(self, records, stream=0):
        """records: list of tuples, one element per ETL provider: HWC uint8 arrays or encoded JPEG
        bytes.  Returns one numpy array per output buffer, shape (n,) + item shape."""
        n = len(records)
        ne = len(self.outputs)
        outs = [np.zeros((n,) + o["shape"], o["dtype"]) for o in self.outputs]
        ptrs = (ctypes.c_void_p * ne)(*[o.ctypes.data for o in outs])
        if any(isinstance(x, (bytes, bytearray, memoryview)) for rec in records for x in rec):
            elems, keep = self._encoded(records)
            _check_host(lib().aeon_decoder_decode_encoded(self._h, n, elems, ptrs, 0, ctypes.c_void_p(stream or 0)))
            return outs
        keep = []
        elems = (RecordElem * (n * ne))()
        for i, rec in enumerate(records):
            for k in range(ne):
                a = np.ascontiguousarray(rec[k], dtype=np.uint8)
                keep.append(a)
                h, w = a.shape[:2]
                cn = 1 if a.ndim == 2 else a.shape[2]
                elems[i * ne + k] = RecordElem(a.ctypes.data, w, h, cn, w * cn)
        _check_host(lib().aeon_decoder_decode(self._h, n, elems, ptrs, 0, ctypes.c_void_p(stream or 0)))
        return outs

    def draw_params(self, sizes, serial=False):
        """The draw phase of one window alone (aeon_decoder_draw_params, host only): sizes = one
        (width, height) per record (of its first element; the others get the same size); returns
        the records' AugParams.  The slot engines advance as in a real window."""
        n, ne = len(sizes), len(self.outputs)
        elems = (RecordElem * (n * ne))()
        dummy = ctypes.c_uint8(0)
        for i, (w, h) in enumerate(sizes):
            for k in range(ne):
                elems[i * ne + k] = RecordElem(ctypes.addressof(dummy), w, h, 3, w * 3)
        out = (AugParams * max(n, 1))()
        _check_host(lib().aeon_decoder_draw_params(self._h, n, elems, out, int(serial)))
        return list(out[:n])

    def submit(self, records, output_ptrs, on_device=False):
        """Double-buffered window (aeon_decoder_submit): output_ptrs[k] = address of n items of
        output k (pinned host memory, or device memory with on_device); complete after wait().
        records: a list of tuples, or an EncodedRecords from encoded() (kept alive by the caller
        until the window's wait())."""
        n, ne = len(records), len(self.outputs)
        elems, keep = self._encoded(records)
        ptrs = (ctypes.c_void_p * ne)(*output_ptrs)
        _check_host(lib().aeon_decoder_submit(self._h, n, elems, ptrs, int(on_device)))

    def wait(self):
        _check_host(lib().aeon_decoder_wait(self._h))

    def pool_cpus(self):
        """Per decode-pool worker: (CPU of the affinity map it was pinned to or -1, the CPUs its own
        sched_getaffinity reported after pinning)."""
        n = ctypes.c_int()
        _check_host(lib().aeon_decoder_pool_size(self._h, ctypes.byref(n)))
        res = []
        for w in range(n.value):
            mc, cnt = ctypes.c_int(), ctypes.c_int()
            buf = (ctypes.c_int * 4096)()
            _check_host(lib().aeon_decoder_pool_cpus(self._h, w, ctypes.byref(mc), buf, 4096, ctypes.byref(cnt)))
            res.append((mc.value, list(buf[:min(cnt.value, 4096)])))
        return res


def thread_affinity_map(cpu_list=""):
    """nervana::get_thread_affinity_map (aeon src/util.cpp:337-373): the CPUs the decode pool's
    workers are pinned to (AEON_CPU_LIST, else cpu_list, else the default policy)."""
    cnt = ctypes.c_int()
    buf = (ctypes.c_int * 4096)()
    _check_host(lib().aeon_thread_affinity_map(cpu_list.encode(), buf, 4096, ctypes.byref(cnt)))
    return list(buf[:min(cnt.value, 4096)])


def manifest_node_slice(record_count, batch_size, node_id, node_count):
    """Record indices of one node (aeon manifest_file node slicing)."""
    cnt = ctypes.c_int64()
    _check_host(lib().aeon_manifest_node_slice(record_count, batch_size, node_id, node_count, None,
                                               ctypes.byref(cnt)))
    out = np.zeros(cnt.value, np.int64)
    _check_host(lib().aeon_manifest_node_slice(record_count, batch_size, node_id, node_count,
                                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                               ctypes.byref(cnt)))
    return out
