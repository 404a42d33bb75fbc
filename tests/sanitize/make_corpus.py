"""Builds tests/sanitize/corpus.npz: malformed JPEG / PNG / JSON inputs for the host parsers.

Seeds are the repo's own small fixtures (tests/golden/jpeg_fixtures.npz, png_fixtures.npz) and the
configuration texts of aeon_amd/configs.py; every mutation is seeded, so the corpus is reproducible:

  python tests/sanitize/make_corpus.py

JPEG: truncations at every segment boundary and inside the scan, random bit flips and byte runs,
over-full / all-ones Huffman tables (the case a fixed overflow in Huffman::build came from), DHT /
DQT / SOF / SOS segment lengths off by one in both directions, sampling factors and table selectors
out of range, zero and oversized frame dimensions, restart intervals, duplicated and dropped segments.
PNG: truncations, bit flips with and without the chunk CRC recomputed (so the mutation reaches
inflate / the row filters), bad IHDR fields, oversized dimensions, palette index overruns.
JSON: truncations, character flips, deep nesting, wrong value types, huge numbers.
"""
import json
import os
import struct
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

JPEG_SEEDS = ["s411_q85.jpg", "gray_rst.jpg", "tiny_3x2.jpg", "narrow_5x300.jpg", "wide_301x4.jpg", "q10.jpg",
              "s420_rst.jpg", "prog_tiny_5x3.jpg", "prog_gray.jpg", "prog_s422_q30.jpg", "s444_rst.jpg"]


def segments(d):
    """(offset of the 0xFF, marker, offset of the length field or None) up to and including SOS."""
    out, p = [], 2
    while p + 4 <= len(d):
        if d[p] != 0xFF:
            break
        m = d[p + 1]
        out.append((p, m, p + 2))
        ln = (d[p + 2] << 8) | d[p + 3]
        if m == 0xDA:
            break
        p += 2 + ln
    return out


def jpeg_mutants(name, d, rng):
    d = bytes(d)
    muts = {}
    segs = segments(d)
    for i, (p, m, lp) in enumerate(segs):  # truncations at and inside each segment
        muts[f"trunc_seg{i}"] = d[:p]
        muts[f"trunc_in_seg{i}"] = d[:lp + 3]
    sos = [s for s in segs if s[1] == 0xDA]
    if sos:
        p = sos[0][0]
        for k, frac in enumerate((0.1, 0.5, 0.9)):
            q = p + int((len(d) - p) * frac)
            muts[f"trunc_scan{k}"] = d[:q]
    for k in range(12):  # random bit flips
        b = bytearray(d)
        for _ in range(int(rng.integers(1, 9))):
            i = int(rng.integers(2, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        muts[f"flip{k}"] = bytes(b)
    for k in range(4):  # runs of 0xFF / 0x00
        b = bytearray(d)
        i = int(rng.integers(2, len(b) - 8))
        b[i:i + 8] = bytes([0xFF if k % 2 else 0x00]) * 8
        muts[f"run{k}"] = bytes(b)
    for i, (p, m, lp) in enumerate(segs):
        ln = (d[lp] << 8) | d[lp + 1]
        for dl, tag in ((1, "p1"), (-1, "m1"), (0x7000, "big"), (-ln + 1, "one"), (-ln, "zero")):
            b = bytearray(d)
            b[lp:lp + 2] = struct.pack(">H", max(0, min(0xFFFF, ln + dl)))
            muts[f"len_{tag}_seg{i}_{m:02x}"] = bytes(b)
        if m == 0xC4:  # DHT: over-full tables with the symbol total kept (the segment still parses)
            counts = list(d[lp + 3:lp + 3 + 16])
            tot = sum(counts)

            def with_counts(c, tag):
                b = bytearray(d)
                b[lp + 3:lp + 3 + 16] = bytes(c)
                muts[f"dht_{tag}_seg{i}"] = bytes(b)

            for short in (1, 2, 9):  # 3 codes of 1 bit (the Huffman::build look[] overflow), 5 of 2, 513 of 9
                need = {1: 3, 2: 5, 9: 513}[short]
                if tot >= need:
                    c = [0] * 16
                    c[short - 1] = min(need, 255)
                    rest = tot - c[short - 1]
                    c[15] = 0
                    for L in range(15, short - 1, -1):  # the remaining symbols at the longest lengths
                        take = min(255, rest)
                        c[L] += take
                        rest -= take
                    if rest == 0:
                        with_counts(c, f"overfull{short}")
            if tot >= 2:  # all-ones code: two 1-bit codes, libjpeg rejects the second
                c = [2] + [0] * 15
                rest = tot - 2
                for L in range(15, 0, -1):
                    take = min(255, rest)
                    c[L] += take
                    rest -= take
                with_counts(c, "allones")
            b = bytearray(d)
            b[lp + 2] = 0x1F  # table class 1, id 15
            muts[f"dht_badid_seg{i}"] = bytes(b)
        if m in (0xC0, 0xC1, 0xC2):  # SOF: sizes, precision, sampling, quant table ids
            for tag, off, val in (("h0", 3, b"\x00\x00"), ("w0", 5, b"\x00\x00"), ("hbig", 3, b"\xff\xff"),
                                  ("wbig", 5, b"\xff\xff"), ("prec12", 2, b"\x0c"), ("ncomp4", 7, b"\x04"),
                                  ("ncomp2", 7, b"\x02"), ("samp0", 9, b"\x00"), ("samp55", 9, b"\x55"),
                                  ("tq9", 10, b"\x09")):
                b = bytearray(d)
                b[lp + off:lp + off + len(val)] = val
                muts[f"sof_{tag}"] = bytes(b)
        if m == 0xDA:  # SOS: component count, selectors, spectral selection
            for tag, off, val in (("ns0", 2, b"\x00"), ("ns4", 2, b"\x04"), ("tsel", 4, b"\xff"),
                                  ("ss", 2 + 1 + 2 * d[lp + 2], b"\x3f\x00"), ("ahal", 2 + 3 + 2 * d[lp + 2], b"\xff")):
                b = bytearray(d)
                if lp + off + len(val) <= len(b):
                    b[lp + off:lp + off + len(val)] = val
                    muts[f"sos_{tag}"] = bytes(b)
            b = bytearray(d)  # SOS whose length field says 2 and the file ends there
            muts["sos_len2_eof"] = bytes(b[:lp]) + b"\x00\x02"
        if m == 0xDD:
            b = bytearray(d)
            b[lp + 2:lp + 4] = b"\x00\x01"
            muts["dri_1"] = bytes(b)
    if len(segs) > 2:  # a segment dropped / duplicated
        p0, _, _ = segs[1]
        p1 = segs[2][0]
        muts["drop_seg1"] = d[:p0] + d[p1:]
        muts["dup_seg1"] = d[:p1] + d[p0:p1] + d[p1:]
    muts["no_soi"] = d[2:]
    muts["only_soi_eoi"] = b"\xff\xd8\xff\xd9"
    muts["empty"] = b""
    return {f"{name[:-4]}__{k}.jpg": v for k, v in muts.items()}


def png_chunks(d):
    out, p = [], 8
    while p + 12 <= len(d):
        ln = struct.unpack(">I", d[p:p + 4])[0]
        out.append((p, d[p + 4:p + 8], ln))
        p += 12 + ln
    return out


def fix_crc(b, p, ln):
    b[p + 8 + ln:p + 12 + ln] = struct.pack(">I", zlib.crc32(bytes(b[p + 4:p + 8 + ln])) & 0xFFFFFFFF)


def png_mutants(name, d, rng):
    d = bytes(d)
    muts = {}
    ch = png_chunks(d)
    for i, (p, t, ln) in enumerate(ch):
        muts[f"trunc_chunk{i}"] = d[:p]
        muts[f"trunc_in_chunk{i}"] = d[:p + 8 + ln // 2]
    for k in range(8):
        b = bytearray(d)
        i = int(rng.integers(8, len(b)))
        b[i] ^= 1 << int(rng.integers(0, 8))
        muts[f"flip{k}"] = bytes(b)
    for k in range(10):  # flips inside a chunk's data with its CRC fixed: the decoder proper runs
        b = bytearray(d)
        p, t, ln = ch[int(rng.integers(0, len(ch)))]
        if ln == 0:
            continue
        for _ in range(int(rng.integers(1, 4))):
            i = p + 8 + int(rng.integers(0, ln))
            b[i] ^= 1 << int(rng.integers(0, 8))
        fix_crc(b, p, ln)
        muts[f"flipcrc{k}_{t.decode('latin1')}"] = bytes(b)
    ihdr = [c for c in ch if c[1] == b"IHDR"]
    if ihdr:
        p, _, ln = ihdr[0]
        for tag, off, val in (("w0", 0, b"\0\0\0\0"), ("wbig", 0, b"\x00\xff\xff\xff"), ("hbig", 4, b"\x7f\xff\xff\xff"),
                              ("depth3", 8, b"\x03"), ("ctype5", 9, b"\x05"), ("interl2", 12, b"\x02"),
                              ("filt1", 11, b"\x01"), ("wide", 0, b"\x00\x00\x40\x00")):
            b = bytearray(d)
            b[p + 8 + off:p + 8 + off + len(val)] = val
            fix_crc(b, p, ln)
            muts[f"ihdr_{tag}"] = bytes(b)
    idat = [c for c in ch if c[1] == b"IDAT"]
    if idat:  # the image data re-deflated with rows cut short / filter bytes out of range
        p, _, ln = idat[0]
        try:
            raw = zlib.decompress(d[p + 8:p + 8 + ln])
        except zlib.error:
            raw = None
        if raw:
            for tag, r in (("short", raw[:len(raw) // 2]), ("badfilter", bytes([7]) + raw[1:]),
                           ("long", raw + raw)):
                z = zlib.compress(r)
                b = bytearray(d[:p]) + struct.pack(">I", len(z)) + b"IDAT" + z + b"\0\0\0\0" + bytearray(d[p + 12 + ln:])
                fix_crc(b, p, len(z))
                muts[f"idat_{tag}"] = bytes(b)
    muts["sig_only"] = d[:8]
    return {f"{name[:-4]}__{k}.png": v for k, v in muts.items()}


def json_mutants(name, text, rng):
    muts = {}
    for k, frac in enumerate((0.0, 0.2, 0.5, 0.8, 0.99)):
        muts[f"trunc{k}"] = text[:int(len(text) * frac)]
    for k in range(10):
        b = bytearray(text.encode())
        i = int(rng.integers(0, len(b)))
        b[i] = int(rng.choice(list(b'{}[]",:0-e.tfn\\ ')))
        muts[f"flip{k}"] = b.decode("latin1")
    muts["deep_arrays"] = "[" * 100000 + "]" * 100000
    muts["deep_objects"] = '{"a":' * 50000 + "1" + "}" * 50000
    muts["deep_unclosed"] = "[" * 200000
    muts["huge_numbers"] = text.replace("0.5", "1e308").replace("1.0", "-1e308")
    muts["nan_like"] = text.replace("0.5", "1e999")
    muts["wrong_types"] = text.replace("[", '"[').replace("]", ']"', 1)
    muts["bad_escape"] = '{"type": "image\\u12"}'
    muts["unterminated"] = '{"type": "ima'
    return {f"{name}__{k}.json": v.encode("latin1") for k, v in muts.items()}


def main():
    rng = np.random.default_rng(2024)
    corpus = {}
    jf = np.load(os.path.join(ROOT, "tests", "golden", "jpeg_fixtures.npz"))
    for n in JPEG_SEEDS:
        d = jf[n].tobytes()
        corpus[f"seed__{n}"] = d
        corpus.update(jpeg_mutants(n, d, rng))
    pf = np.load(os.path.join(ROOT, "tests", "golden", "png_fixtures.npz"))
    pngs = sorted(k for k in pf.keys() if k.endswith(".png"))
    for n in pngs[::3]:
        d = pf[n].tobytes()
        corpus[f"seed__{n}"] = d
        corpus.update(png_mutants(n, d, rng))
    from aeon_amd import configs as C
    for nm in ("C1_AUG", "C2_AUG", "C3_AUG", "C5_AUG"):
        text = json.dumps(getattr(C, nm))
        corpus[f"seed__{nm}.json"] = text.encode()
        corpus.update(json_mutants(nm, text, rng))
    np.savez_compressed(os.path.join(HERE, "corpus.npz"),
                        **{k: np.frombuffer(v, np.uint8) for k, v in corpus.items()})
    print(len(corpus), "inputs,", sum(len(v) for v in corpus.values()), "bytes")


if __name__ == "__main__":
    main()
