"""Test infrastructure only (tests/ may import it; the product never does): a plain Python + numpy
restatement of cv::imdecode on PNG files as aeon's extractors call it (src/etl_image.cpp:83-99
CV_LOAD_IMAGE_COLOR / GRAYSCALE, src/etl_pixel_mask.cpp:30-53 CV_LOAD_IMAGE_ANYDEPTH), i.e. OpenCV
2.4's PngDecoder over libpng:
  * PNG itself (ISO/IEC 15948): chunk walk with CRC checks of critical chunks, zlib inflate of the
    IDAT stream, the five row filters, Adam7 interlacing, 1/2/4/8/16-bit samples;
  * the libpng transforms OpenCV requests: strip alpha, palette -> RGB, 1/2/4-bit gray expanded
    to 8 bits, RGB -> BGR (colour) or rgb_to_gray(1, 0.299, 0.587) with libpng's truncating 15-bit
    fixed point (gray), 16 -> 8 bits by the high byte unless ANYDEPTH keeps 16-bit gray.
Pinned by tests/golden/png_fixtures.npz (files encoded from known pixels, and Pillow-written files
whose Pillow decode matches); the libpng colour reductions themselves are parity unpinned (libpng
and OpenCV are absent here).
"""
import struct
import zlib

import numpy as np

BGR8, GRAY8, ANYDEPTH = 0, 1, 2
_RC, _GC = 29900 * 32768 // 100000, 58700 * 32768 // 100000
_BC = 32768 - _RC - _GC
_SAMPLES = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}
_ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


class PngError(ValueError):
    pass


def _chunks(data):
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise PngError("bad signature")
    p = 8
    while p + 12 <= len(data):
        n, t = struct.unpack(">I4s", data[p:p + 8])
        body = data[p + 8:p + 8 + n]
        if len(body) != n or p + 12 + n > len(data):
            raise PngError("truncated chunk")
        crc = struct.unpack(">I", data[p + 8 + n:p + 12 + n])[0]
        if not (t[0] & 0x20) and zlib.crc32(t + body) & 0xFFFFFFFF != crc:
            raise PngError("CRC error")
        yield t, body
        if t == b"IEND":
            return
        p += 12 + n


def _unfilter(buf, w, h, bits):
    rowb, bpp = (w * bits + 7) // 8, max(1, bits // 8)
    out = np.zeros((h, rowb), np.int64)
    for y in range(h):
        ft, line = buf[y * (rowb + 1)], np.frombuffer(buf, np.uint8, rowb, y * (rowb + 1) + 1).astype(np.int64)
        up = out[y - 1] if y else np.zeros(rowb, np.int64)
        if ft == 0:
            out[y] = line
        elif ft == 2:
            out[y] = (line + up) & 255
        elif ft in (1, 3, 4):
            cur = out[y]
            for i in range(rowb):
                a = cur[i - bpp] if i >= bpp else 0
                b = up[i]
                c = up[i - bpp] if i >= bpp else 0
                if ft == 1:
                    pred = a
                elif ft == 3:
                    pred = (a + b) // 2
                else:
                    pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                    pred = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                cur[i] = (line[i] + pred) & 255
        else:
            raise PngError("bad filter")
    return out


def _samples(rows, w, n, depth):
    """packed rows (h, rowb) -> (h, w*n) sample values"""
    if depth == 8:
        return rows[:, :w * n]
    if depth == 16:
        return (rows[:, 0:2 * w * n:2] << 8) | rows[:, 1:2 * w * n:2]
    per = 8 // depth
    shifts = np.array([8 - depth * (k + 1) for k in range(per)])
    v = (rows[:, :, None] >> shifts) & ((1 << depth) - 1)
    return v.reshape(rows.shape[0], -1)[:, :w * n]


def decode(data, mode=BGR8):
    """-> HxWx3 uint8 (BGR8) / HxW uint8 (GRAY8) / HxW uint8 or uint16 (ANYDEPTH)"""
    hdr, pal, idat = None, None, b""
    for t, body in _chunks(bytes(data)):
        if t == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif t == b"PLTE":
            pal = np.frombuffer(body, np.uint8).reshape(-1, 3).astype(np.int64)
        elif t == b"IDAT":
            idat += body
    if hdr is None:
        raise PngError("no IHDR")
    w, h, depth, ctype, _, _, interlace = hdr
    n = _SAMPLES[ctype]
    raw = zlib.decompress(idat)
    img = np.zeros((h, w, n), np.int64)
    passes = _ADAM7 if interlace else [(0, 0, 1, 1)]
    off = 0
    for x0, y0, dx, dy in passes:
        pw, ph = (w - x0 + dx - 1) // dx, (h - y0 + dy - 1) // dy
        if pw <= 0 or ph <= 0:
            continue
        size = ph * ((pw * n * depth + 7) // 8 + 1)
        rows = _unfilter(raw[off:off + size], pw, ph, n * depth)
        img[y0::dy, x0::dx] = _samples(rows, pw, n, depth).reshape(ph, pw, n)
        off += size
    if ctype == 3:
        rgb, d = pal[img[:, :, 0]], 8
    elif ctype in (0, 4):
        v = img[:, :, 0] * ({1: 255, 2: 85, 4: 17}.get(depth, 1))
        rgb, d = np.stack([v, v, v], -1), max(depth, 8)
    else:
        rgb, d = img[:, :, :3], depth
    r, g, b = rgb[:, :, 0], rgb[:, :, 1], rgb[:, :, 2]
    if mode == BGR8:
        return (np.stack([b, g, r], -1) >> (8 if d == 16 else 0)).astype(np.uint8)
    gray = np.where((r == g) & (r == b), r, (_RC * r + _GC * g + _BC * b) >> 15)
    if mode == ANYDEPTH and d == 16:
        return gray.astype(np.uint16)
    return (gray >> (8 if d == 16 else 0)).astype(np.uint8)
