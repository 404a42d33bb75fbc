"""Generate the committed JPEG-decode golden fixtures (image::extractor::extract, aeon
src/etl_image.cpp:83-99 -> cv::imdecode -> libjpeg).

Run in the dev container only (reads /root/reference and uses Pillow); the output is committed so
tests never touch the reference.  Expected values are Pillow 12.2 / libjpeg-turbo decodes -- the
ISLOW IDCT + fancy-upsampling decoder settings OpenCV's imdecode uses (the same decoder that
reproduces aeon's augment_output_linear goldens from img_2112_70.jpg, tests/golden/make_fixtures.py).

jpeg_fixtures.npz, per fixture <name>:
  <name>.jpg     the file's bytes (uint8)
  <name>.bgr     sha256 of the HWC BGR decode (cv::imdecode(..., CV_LOAD_IMAGE_COLOR))
  <name>.gray    sha256 of the grayscale decode (CV_LOAD_IMAGE_GRAYSCALE: the Y component)
  <name>.shape   (height, width)
  <name>.bgr_px  the full BGR decode, for the small synthetic fixtures only
Fixtures: aeon's own test/test_data/img_2112_70.jpg and flowers.jpg (4:2:0 baseline), and files
Pillow encodes from seeded smooth-noise images: 4:4:4 / 4:2:2 / 4:2:0 / 4:1:1, grayscale, restart
intervals, sizes from 1x1 up, qualities 10..100, and progressive files (synthetic ones and aeon's two
images re-encoded progressive).
"""
import hashlib
import io
import os
import sys

import numpy as np

REF = "/root/reference/test/test_data"
HERE = os.path.dirname(os.path.abspath(__file__))


def _sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def _decode(b):
    from PIL import Image
    bgr = np.ascontiguousarray(np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))[:, :, ::-1])
    im = Image.open(io.BytesIO(b))
    im.draft("L", im.size)  # libjpeg JCS_GRAYSCALE output: the Y component
    gray = np.asarray(im if im.mode == "L" else im.convert("L"))
    return bgr, gray


def synthetic():
    from PIL import Image
    rng = np.random.default_rng(2024)
    cases = [  # (name, w, h, mode, subsampling, quality, restart blocks)
        ("s444_q90", 97, 61, "RGB", "4:4:4", 90, 0), ("s422_q75", 130, 77, "RGB", "4:2:2", 75, 0),
        ("s420_q50", 225, 129, "RGB", "4:2:0", 50, 0), ("s411_q85", 71, 33, "RGB", "4:1:1", 85, 0),
        ("s420_rst", 161, 95, "RGB", "4:2:0", 80, 3), ("s444_rst", 40, 40, "RGB", "4:4:4", 95, 1),
        ("gray_q70", 123, 45, "L", None, 70, 0), ("gray_rst", 64, 64, "L", None, 30, 2),
        ("tiny_1x1", 1, 1, "RGB", "4:2:0", 90, 0), ("tiny_3x2", 3, 2, "RGB", "4:2:0", 90, 0),
        ("narrow_5x300", 5, 300, "RGB", "4:2:0", 60, 0), ("wide_301x4", 301, 4, "RGB", "4:2:2", 60, 0),
        ("q100", 80, 72, "RGB", "4:2:0", 100, 0), ("q10", 88, 56, "RGB", "4:2:0", 10, 0),
        # progressive (SOF2: spectral selection + successive approximation scans)
        ("prog_s420", 150, 110, "RGB", "4:2:0", 85, 0), ("prog_s444_rst", 90, 70, "RGB", "4:4:4", 90, 2),
        ("prog_gray", 77, 51, "L", None, 75, 0), ("prog_s422_q30", 131, 67, "RGB", "4:2:2", 30, 0),
        ("prog_q100", 64, 48, "RGB", "4:2:0", 100, 0), ("prog_tiny_5x3", 5, 3, "RGB", "4:2:0", 90, 0),
    ]
    out = []
    for name, w, h, mode, sub, q, rst in cases:
        base = rng.integers(0, 256, (h // 8 + 2, w // 8 + 2, 3)).astype(np.uint8)
        arr = np.asarray(Image.fromarray(base).resize((w, h), Image.BILINEAR)).astype(np.int32)
        arr = np.clip(arr + rng.integers(-40, 40, arr.shape), 0, 255).astype(np.uint8)
        im = Image.fromarray(arr if mode == "RGB" else arr[:, :, 0])
        kw = {"quality": q}
        if sub:
            kw["subsampling"] = sub
        if rst:
            kw["restart_marker_blocks"] = rst
        if name.startswith("prog_"):
            kw["progressive"] = True
        bio = io.BytesIO()
        im.save(bio, "JPEG", **kw)
        out.append((name, bio.getvalue(), True))
    return out


def main():
    files = [(n[:-4], open(os.path.join(REF, n), "rb").read(), False) for n in ("img_2112_70.jpg", "flowers.jpg")]
    files += synthetic()
    # aeon's two test images re-encoded progressive (from their baseline decode, Pillow quality 90)
    from PIL import Image
    for n, (_, src, _) in zip(("img_2112_70", "flowers"), files[:2]):
        bio = io.BytesIO()
        Image.open(io.BytesIO(src)).save(bio, "JPEG", quality=90, progressive=True)
        files.append(("prog_" + n, bio.getvalue(), False))
    fx = {}
    for name, b, keep in files:
        bgr, gray = _decode(b)
        fx[name + ".jpg"] = np.frombuffer(b, np.uint8)
        fx[name + ".bgr"] = _sha(bgr)
        fx[name + ".gray"] = _sha(gray)
        fx[name + ".shape"] = np.array(gray.shape, np.int32)
        if keep:
            fx[name + ".bgr_px"] = bgr
    np.savez_compressed(os.path.join(HERE, "jpeg_fixtures.npz"), **fx)
    print(len(files), "JPEG fixtures written to", HERE)


if __name__ == "__main__":
    sys.exit(main())
