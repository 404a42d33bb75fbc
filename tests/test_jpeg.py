"""JPEG decode -- image::extractor::extract (aeon src/etl_image.cpp:83-99: cv::imdecode -> libjpeg
ISLOW + fancy upsampling, BGR / grayscale output).

CPU: the oracle restatement (oracle/jpeg_oracle.cpp) against the committed goldens
(tests/golden/make_jpeg_fixtures.py: Pillow/libjpeg-turbo decodes of aeon's own
test/test_data/img_2112_70.jpg and flowers.jpg plus Pillow-encoded files), and the product's header
parser (aeon_jpeg_info).  GPU: the product's decode (aeon_hip_decode_jpeg_batch: sequential files
entropy-decoded on the GPU by jpeg_huff, progressive ones on the host pool, then the IDCT / upsampling /
colour kernels) bit-exact against the same goldens and the oracle, and the GPU entropy decoder against
the host one (AEON_HIP_JPEG_HUFF=host) file for file.
"""
import hashlib
import os

import numpy as np
import pytest

import aeon_amd as A

HERE = os.path.dirname(os.path.abspath(__file__))
FX = np.load(os.path.join(HERE, "golden", "jpeg_fixtures.npz"))
NAMES = sorted({k.rsplit(".", 1)[0] for k in FX.files})


def _sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def _jpg(name):
    return FX[name + ".jpg"].tobytes()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_jpeg_matches_golden(oracle, name):
    b = _jpg(name)
    h, w = FX[name + ".shape"]
    bgr = oracle.jpeg_decode(b, 3)
    assert bgr.shape == (h, w, 3)
    if name + ".bgr_px" in FX.files:
        assert np.array_equal(bgr, FX[name + ".bgr_px"])
    assert np.array_equal(_sha(bgr), FX[name + ".bgr"]), name
    assert np.array_equal(_sha(oracle.jpeg_decode(b, 1)), FX[name + ".gray"]), name


def test_oracle_jpeg_img_2112_70_is_the_golden_source(oracle):
    """The decode that feeds aeon's augment goldens (tests/golden/img_2112_70_bgr.npz)."""
    ref = np.load(os.path.join(HERE, "golden", "img_2112_70_bgr.npz"))["bgr"]
    assert np.array_equal(oracle.jpeg_decode(_jpg("img_2112_70"), 3), ref)


@pytest.mark.parametrize("name", NAMES)
def test_product_jpeg_info(oracle, name):
    b = _jpg(name)
    h, w = FX[name + ".shape"]
    assert A.jpeg_info(b)[:2] == (w, h)
    assert A.jpeg_info(b) == oracle.jpeg_info(b)


def test_product_jpeg_info_rejects_garbage():
    with pytest.raises(A.AeonHipError):
        A.jpeg_info(b"\x00\x01not a jpeg")
    b = _jpg("img_2112_70")
    with pytest.raises(A.AeonHipError):
        A.jpeg_info(b[:100])  # truncated before the frame header ends


def _mcu_too_large(name="s444_q90"):
    """The file with every component's sampling factors set to 2x2 in its SOF0: 12 blocks per MCU of
    its interleaved scan, past libjpeg's D_MAX_BLOCKS_IN_MCU (10)."""
    b = bytearray(_jpg(name))
    i = b.index(b"\xff\xc0")
    ncomp = b[i + 9]
    assert ncomp == 3
    for k in range(ncomp):
        b[i + 11 + 3 * k] = 0x22
    return bytes(b)


def test_interleaved_mcu_over_ten_blocks_refused(oracle):
    """libjpeg (jdinput.c per_scan_setup) refuses an interleaved scan of more than 10 blocks per MCU with
    JERR_BAD_MCU_SIZE, so cv::imdecode -- aeon's extract -- fails on such a file: the product's host stage
    and host entropy decoder and the oracle refuse it too (the header alone still parses)."""
    b = _mcu_too_large()
    assert A.jpeg_info(b)[2] == 3
    for fn in (A.jpeg_entropy_decode, A.jpeg_host_stage):
        with pytest.raises(A.AeonHipError, match="sampling factors too large"):
            fn(b)
    with pytest.raises(Exception, match="sampling factors too large"):
        oracle.jpeg_decode(b)


def _decode_gpu(ctx, files, channels):
    import torch
    infos = [A.jpeg_info(b) for b in files]
    descs, off = [], 0
    for (w, h, _) in infos:
        descs.append(A.ImgDesc(offset=off, width=w, height=h, stride=w * channels, channels=channels))
        off += (w * h * channels + 15) // 16 * 16
    dst = torch.full((max(off, 16),), 0x5A, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ctx.decode_jpeg_batch(files, descs, dst.data_ptr(), stream)
    ctx.synchronize(stream)
    host = dst.cpu().numpy()
    out = []
    for d in descs:
        a = host[d.offset:d.offset + d.width * d.height * channels]
        out.append(a.reshape(d.height, d.width, channels) if channels == 3 else a.reshape(d.height, d.width))
    return out


@pytest.fixture(scope="module")
def ctx():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    c = A.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("channels", [3, 1])
def test_gpu_jpeg_batch_matches_golden(ctx, oracle, channels):
    files = [_jpg(n) for n in NAMES]
    res = _decode_gpu(ctx, files, channels)
    for name, b, r in zip(NAMES, files, res):
        want = FX[name + (".bgr" if channels == 3 else ".gray")]
        if not np.array_equal(_sha(r), want):
            ref = oracle.jpeg_decode(b, channels)
            bad = np.argwhere(r != ref)
            raise AssertionError(f"{name}: {len(bad)} mismatches vs oracle, first {bad[:3].tolist()}")


@pytest.mark.gpu
@pytest.mark.parametrize("band", [1, 2, 3, 8])
def test_gpu_jpeg_colour_bands(ctx, band, monkeypatch):
    """The colour pass with short bands of output rows per workgroup (AEON_HIP_JPEG_BAND; the default
    is 32): odd band starts take the general path, even ones the 4:2:0 row-pair path with a band
    that ends on an odd row -- every fixture still matches its golden digest."""
    monkeypatch.setenv("AEON_HIP_JPEG_BAND", str(band))
    files = [_jpg(n) for n in NAMES]
    res = _decode_gpu(ctx, files, 3)
    for name, r in zip(NAMES, res):
        assert np.array_equal(_sha(r), FX[name + ".bgr"]), (name, band)


@pytest.mark.gpu
def test_gpu_jpeg_large_batch_repeatable(ctx, oracle):
    """A decode window of 300 JPEGs (the two aeon fixtures cycled with the synthetic ones):
    bit-exact against the oracle and identical on a rerun."""
    files = [_jpg(NAMES[i % len(NAMES)]) for i in range(300)]
    r1 = _decode_gpu(ctx, files, 3)
    r2 = _decode_gpu(ctx, files, 3)
    for i, (a, b) in enumerate(zip(r1, r2)):
        assert np.array_equal(a, b), i
    cache = {}
    for i, b in enumerate(files):
        if b not in cache:
            cache[b] = oracle.jpeg_decode(b, 3)
        assert np.array_equal(r1[i], cache[b]), i


@pytest.mark.gpu
def test_gpu_jpeg_errors(ctx):
    import torch
    dst = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    b = _jpg("tiny_3x2")
    with pytest.raises(A.AeonHipError, match="does not match"):
        ctx.decode_jpeg_batch([b], [A.ImgDesc(offset=0, width=4, height=2, stride=12, channels=3)], dst.data_ptr())
    with pytest.raises(A.AeonHipError):
        ctx.decode_jpeg_batch([b[:40]], [A.ImgDesc(offset=0, width=3, height=2, stride=9, channels=3)],
                              dst.data_ptr())


@pytest.fixture(scope="module")
def host_ctx():
    """A context whose JPEG stage entropy-decodes every file on the host (the flag is read when the
    context is created)."""
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    os.environ["AEON_HIP_JPEG_HUFF"] = "host"
    try:
        c = A.Context(0)
    finally:
        del os.environ["AEON_HIP_JPEG_HUFF"]
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("channels", [3, 1])
def test_gpu_huffman_matches_host_huffman(ctx, host_ctx, channels):
    """Every fixture through the GPU entropy decoder (jpeg_huff) and through the host one: the same
    decoded records, in one mixed call (sequential, restart-interval and progressive files together)."""
    files = [_jpg(n) for n in NAMES] * 3
    a = _decode_gpu(ctx, files, channels)
    b = _decode_gpu(host_ctx, files, channels)
    for i, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), NAMES[i % len(NAMES)]


@pytest.mark.gpu
def test_gpu_huffman_window_of_aeon_files(ctx, oracle):
    """A bench-sized window (256 records: aeon's img_2112_70.jpg and flowers.jpg alternating) through
    the GPU entropy decoder: bit-exact against the oracle's decode of each file."""
    files = [_jpg("img_2112_70"), _jpg("flowers")] * 128
    res = _decode_gpu(ctx, files, 3)
    want = [oracle.jpeg_decode(files[0], 3), oracle.jpeg_decode(files[1], 3)]
    for i, r in enumerate(res):
        assert np.array_equal(r, want[i % 2]), i


@pytest.mark.gpu
def test_gpu_huffman_corrupt_data_reported(ctx):
    """Corrupt entropy-coded data of a GPU-decoded file (a flipped scan byte: an invalid Huffman code,
    and a scan cut off with the file) comes back from aeon_hip_synchronize as a device error, and the
    context decodes the next good window normally."""
    import torch
    # two inputs of tests/sanitize/corpus.npz (make_corpus.py), kept in tests/golden for the GPU box
    corpus = np.load(os.path.join(HERE, "golden", "jpeg_corrupt.npz"))
    for bad in ("s411_q85__flip10.jpg", "gray_rst__trunc_scan0.jpg"):
        b = corpus[bad].tobytes()
        w, h, n = A.jpeg_info(b)
        dst = torch.zeros(w * h * 3 + 16, dtype=torch.uint8, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        ctx.decode_jpeg_batch([b], [A.ImgDesc(offset=0, width=w, height=h, stride=w * 3, channels=3)],
                              dst.data_ptr(), stream)
        with pytest.raises(A.AeonHipError, match="JPEG entropy-coded data corrupt"):
            ctx.synchronize(stream)
    good = [_jpg("s420_q50")]
    r = _decode_gpu(ctx, good, 3)
    assert np.array_equal(_sha(r[0]), FX["s420_q50.bgr"])
