"""PNG decode -- image::extractor::extract / pixel_mask::extractor::extract on PNG files (aeon
src/etl_image.cpp:83-99, src/etl_pixel_mask.cpp:30-53: cv::imdecode over libpng).  Host code in
the product (png_host.cpp, aeon_decode_png), so these run on the CPU: the oracle restatement
(oracle/png_oracle.py) and the product against the committed fixtures
(tests/golden/make_png_fixtures.py: files encoded from known pixels over every colour type, bit
depth, row filter and Adam7, plus Pillow-written files) and against each other on random files.
The libpng colour reductions (rgb_to_gray, strip_16) are parity unpinned (no libpng here).
"""
import io
import os
import struct
import zlib

import numpy as np
import pytest

import aeon_amd as A
from oracle import png_oracle as PO

HERE = os.path.dirname(os.path.abspath(__file__))
FX = np.load(os.path.join(HERE, "golden", "png_fixtures.npz"))
NAMES = sorted({k.rsplit(".", 1)[0] for k in FX.files})
MODES = [(A.PNG_BGR8, "bgr8"), (A.PNG_GRAY8, "gray8"), (A.PNG_ANYDEPTH, "any")]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_png_matches_fixture(name):
    png = FX[name + ".png"].tobytes()
    for mode, key in MODES:
        out = PO.decode(png, mode)
        assert out.dtype == FX[name + "." + key].dtype and np.array_equal(out, FX[name + "." + key]), (name, key)


@pytest.mark.parametrize("name", NAMES)
def test_product_png_matches_fixture(name):
    png = FX[name + ".png"].tobytes()
    w, h, depth, ctype = A.png_info(png)
    assert (h, w) == FX[name + ".gray8"].shape
    for mode, key in MODES:
        out = A.decode_png(png, mode)
        assert out.dtype == FX[name + "." + key].dtype and np.array_equal(out, FX[name + "." + key]), (name, key)


def test_product_png_matches_oracle_random():
    from PIL import Image
    rng = np.random.default_rng(5)
    for i in range(24):
        mode = ["RGB", "L", "RGBA", "P", "I;16", "LA"][i % 6]
        h, w = int(rng.integers(1, 40)), int(rng.integers(1, 40))
        if mode == "I;16":
            arr = rng.integers(0, 65536, (h, w)).astype(np.uint16)
            im = Image.fromarray(arr)
        elif mode == "P":
            im = Image.fromarray(rng.integers(0, 64, (h, w)).astype(np.uint8), "P")
            im.putpalette(rng.integers(0, 256, 64 * 3).tolist())
        else:
            shape = {"RGB": (h, w, 3), "L": (h, w), "RGBA": (h, w, 4), "LA": (h, w, 2)}[mode]
            im = Image.fromarray(rng.integers(0, 256, shape).astype(np.uint8), mode)
        buf = io.BytesIO()
        im.save(buf, "PNG", optimize=bool(i % 2))
        png = buf.getvalue()
        for m, _ in MODES:
            a, b = A.decode_png(png, m), PO.decode(png, m)
            assert a.dtype == b.dtype and np.array_equal(a, b), (mode, m)


def _corrupt(png, at, value):
    b = bytearray(png)
    b[at] = value
    return bytes(b)


def test_png_errors():
    png = FX["gray8_n.png"].tobytes()
    with pytest.raises(A.AeonHipError):
        A.png_info(b"\x89PNX" + png[4:])
    # a flipped byte inside IHDR breaks its CRC (libpng: error on a critical chunk)
    with pytest.raises(A.AeonHipError) as e:
        A.decode_png(_corrupt(png, 18, png[18] ^ 1))
    assert "CRC" in str(e.value)
    with pytest.raises(A.AeonHipError):
        A.decode_png(png[:60])
    with pytest.raises(A.AeonHipError):
        A.decode_png(png, 7)
    # an IDAT stream too short for the image
    ihdr = struct.pack(">IIBBBBB", 8, 8, 8, 0, 0, 0, 0)
    z = zlib.compress(b"\x00" * 9 * 4)

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    short = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", z) + chunk(b"IEND", b"")
    with pytest.raises(A.AeonHipError):
        A.decode_png(short)
    with pytest.raises(PO.PngError):
        PO.decode(_corrupt(png, 18, png[18] ^ 1))
