"""Generate tests/golden/png_fixtures.npz: PNG files and what aeon's extractors decode them to.

Two kinds of file:
  * written here by a small PNG encoder (numpy + zlib) from KNOWN pixels, covering every colour
    type, every bit depth, the five row filters (row y uses filter y % 5), Adam7 interlacing, a
    split IDAT stream and a tRNS chunk;
  * written by Pillow (its own encoder and filter choice), whose decode Pillow also provides.
Expected outputs follow the cv::imdecode-over-libpng semantics (png_host.cpp header) from the
known pixels: BGR8 (CV_LOAD_IMAGE_COLOR), GRAY8 (CV_LOAD_IMAGE_GRAYSCALE) and ANYDEPTH
(CV_LOAD_IMAGE_ANYDEPTH, masks).  For Pillow-written files the decoded pixels are Pillow's and are
checked against the known source before use.

Run once, in the dev container: python tests/golden/make_png_fixtures.py
"""
import io
import os
import struct
import zlib

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
RC, GC = 29900 * 32768 // 100000, 58700 * 32768 // 100000
BC = 32768 - RC - GC
ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def chunk(t, data):
    return struct.pack(">I", len(data)) + t + data + struct.pack(">I", zlib.crc32(t + data) & 0xFFFFFFFF)


def pack_rows(samples, depth):
    """samples: (h, n) ints -> list of packed row byte strings."""
    rows = []
    for r in samples:
        if depth == 16:
            rows.append(b"".join(struct.pack(">H", int(v)) for v in r))
        elif depth == 8:
            rows.append(bytes(int(v) for v in r))
        else:
            bits = "".join(format(int(v), "0%db" % depth) for v in r)
            bits += "0" * (-len(bits) % 8)
            rows.append(bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8)))
    return rows


def filter_rows(rows, bpp):
    out, prev = [], None
    for y, row in enumerate(rows):
        ft = y % 5
        a = [row[i - bpp] if i >= bpp else 0 for i in range(len(row))]
        b = list(prev) if prev is not None else [0] * len(row)
        c = [prev[i - bpp] if (prev is not None and i >= bpp) else 0 for i in range(len(row))]
        f = []
        for i, x in enumerate(row):
            if ft == 0:
                p = 0
            elif ft == 1:
                p = a[i]
            elif ft == 2:
                p = b[i]
            elif ft == 3:
                p = (a[i] + b[i]) >> 1
            else:
                pp = a[i] + b[i] - c[i]
                pa, pb, pc = abs(pp - a[i]), abs(pp - b[i]), abs(pp - c[i])
                p = a[i] if (pa <= pb and pa <= pc) else (b[i] if pb <= pc else c[i])
            f.append((x - p) & 255)
        out.append(bytes([ft]) + bytes(f))
        prev = row
    return b"".join(out)


def encode(px, depth, ctype, palette=None, interlace=False, trns=None):
    """px: (h, w, samples) ints at `depth`."""
    h, w, s = px.shape
    bpp = max(1, s * depth // 8)
    raw = b""
    if interlace:
        for x0, y0, dx, dy in ADAM7:
            sub = px[y0::dy, x0::dx]
            if sub.shape[0] and sub.shape[1]:
                raw += filter_rows(pack_rows(sub.reshape(sub.shape[0], -1), depth), bpp)
    else:
        raw = filter_rows(pack_rows(px.reshape(h, -1), depth), bpp)
    z = zlib.compress(raw, 6)
    out = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, int(interlace)))
    if palette is not None:
        out += chunk(b"PLTE", bytes(np.asarray(palette, np.uint8).reshape(-1)))
    if trns is not None:
        out += chunk(b"tRNS", trns)
    out += chunk(b"tEXt", b"Comment\x00aeon fixture")  # an ancillary chunk to skip
    half = len(z) // 2
    out += chunk(b"IDAT", z[:half]) + chunk(b"IDAT", z[half:]) + chunk(b"IEND", b"")
    return out


def expected(px, depth, ctype, palette=None):
    """(bgr8, gray8, anydepth) from the known pixels."""
    px = px.astype(np.int64)
    if ctype == 3:
        rgb = np.asarray(palette, np.int64)[px[:, :, 0]]
        d = 8
    elif ctype in (0, 4):
        v = px[:, :, 0]
        if depth < 8:
            v = v * {1: 255, 2: 85, 4: 17}[depth]
        rgb = np.stack([v, v, v], -1)
        d = max(depth, 8)
    else:
        rgb = px[:, :, :3]
        d = depth
    r, g, b = rgb[:, :, 0], rgb[:, :, 1], rgb[:, :, 2]
    bgr8 = (np.stack([b, g, r], -1) >> (8 if d == 16 else 0)).astype(np.uint8)
    gray = np.where((r == g) & (r == b), r, (RC * r + GC * g + BC * b) >> 15)
    gray8 = (gray >> (8 if d == 16 else 0)).astype(np.uint8)
    anyd = gray.astype(np.uint16) if d == 16 else gray.astype(np.uint8)
    return bgr8, gray8, anyd


def main():
    rng = np.random.default_rng(2024)
    fx = {}

    def add(name, png, px, depth, ctype, palette=None):
        b8, g8, ad = expected(px, depth, ctype, palette)
        fx[name + ".png"] = np.frombuffer(png, np.uint8)
        fx[name + ".bgr8"], fx[name + ".gray8"], fx[name + ".any"] = b8, g8, ad

    sizes = [(1, 1), (3, 5), (17, 33), (24, 19)]
    for interlace in (False, True):
        tag = "i" if interlace else "n"
        for depth in (1, 2, 4, 8, 16):  # gray
            h, w = sizes[depth % len(sizes)] if depth != 8 else (24, 19)
            px = rng.integers(0, 1 << depth, (h, w, 1))
            add(f"gray{depth}_{tag}", encode(px, depth, 0, interlace=interlace), px, depth, 0)
        for depth in (8, 16):  # RGB, gray+alpha, RGBA
            for ctype, s in ((2, 3), (4, 2), (6, 4)):
                h, w = (13, 21) if depth == 8 else (9, 11)
                px = rng.integers(0, 1 << depth, (h, w, s))
                if ctype == 2:  # some grey pixels: rgb_to_gray keeps them
                    px[0, :, 1] = px[0, :, 2] = px[0, :, 0]
                add(f"c{ctype}_{depth}_{tag}", encode(px, depth, ctype, interlace=interlace), px, depth, ctype)
        for depth in (1, 2, 4, 8):  # palette
            n = 1 << depth
            pal = rng.integers(0, 256, (n, 3))
            pal[0] = (7, 7, 7)
            h, w = (10, 23)
            px = rng.integers(0, n, (h, w, 1))
            trns = bytes([0, 128]) if depth == 2 else None
            add(f"pal{depth}_{tag}", encode(px, depth, 3, palette=pal, interlace=interlace, trns=trns), px, depth, 3,
                pal)
    # Pillow-written files (Pillow's encoder and filters); Pillow's decode equals the source
    for name, arr, mode in [("pil_rgb", rng.integers(0, 256, (31, 45, 3)), "RGB"),
                            ("pil_l", rng.integers(0, 256, (29, 40)), "L"),
                            ("pil_rgba", rng.integers(0, 256, (16, 20, 4)), "RGBA")]:
        im = Image.fromarray(arr.astype(np.uint8), mode)
        buf = io.BytesIO()
        im.save(buf, "PNG", optimize=True)
        png = buf.getvalue()
        back = np.asarray(Image.open(io.BytesIO(png)))
        assert np.array_equal(back, arr), name
        px = arr.reshape(arr.shape[0], arr.shape[1], -1)
        add(name, png, px, 8, {"RGB": 2, "L": 0, "RGBA": 6}[mode])
    arr16 = rng.integers(0, 65536, (12, 17)).astype(np.uint16)
    im = Image.fromarray(arr16)  # 16-bit gray ("I;16")
    buf = io.BytesIO()
    im.save(buf, "PNG")
    png = buf.getvalue()
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(png))).astype(np.uint16), arr16)
    add("pil_gray16", png, arr16.reshape(12, 17, 1).astype(np.int64), 16, 0)
    pal = rng.integers(0, 256, (200, 3)).astype(np.uint8)
    idx = rng.integers(0, 200, (14, 27)).astype(np.uint8)
    im = Image.fromarray(idx, "P")
    im.putpalette(pal.reshape(-1).tolist())
    buf = io.BytesIO()
    im.save(buf, "PNG")
    png = buf.getvalue()
    assert np.array_equal(np.asarray(Image.open(io.BytesIO(png))), idx)
    add("pil_pal", png, idx.reshape(14, 27, 1).astype(np.int64), 8, 3, pal.astype(np.int64))
    np.savez_compressed(os.path.join(HERE, "png_fixtures.npz"), **fx)
    print(len(fx) // 4, "PNG fixtures")


if __name__ == "__main__":
    main()
