// png_host.cpp -- the PNG half of image::extractor::extract / pixel_mask::extractor::extract (aeon
// src/etl_image.cpp:83-99, src/etl_pixel_mask.cpp:30-53): cv::imdecode over libpng, restated on
// zlib's inflate.  Host code by nature: inflate is a serial bit stream and the PNG row filters
// (Sub / Up / Average / Paeth) chain every row to the one above and every pixel to the one on its
// left, so a record decodes on one decode-pool thread straight into the pinned staging arena.
//
// Output forms (what OpenCV 2.4's PngDecoder asks libpng for):
//   AEON_PNG_BGR8   -- CV_LOAD_IMAGE_COLOR: 8-bit BGR.  16-bit samples keep their high byte
//                      (png_set_strip_16), 1/2/4-bit gray expands to 8 bits (x 255 / 85 / 17),
//                      palettes expand to RGB, gray replicates to three channels, alpha is dropped.
//   AEON_PNG_GRAY8  -- CV_LOAD_IMAGE_GRAYSCALE: 8-bit gray; colour goes through libpng's
//                      png_set_rgb_to_gray(1, 0.299, 0.587): 15-bit coefficients 9797 / 19234 /
//                      3737, truncating, and a pixel with R == G == B keeps its value.
//   AEON_PNG_ANYDEPTH -- CV_LOAD_IMAGE_ANYDEPTH (pixel masks, depth maps): gray at the file's depth,
//                      8 or 16 bits (16-bit samples as native uint16), colour reduced as above.
// Adam7 interlacing, every colour type and bit depth, and CRC checks of the critical chunks are
// handled; tRNS only feeds alpha, which every form drops.
#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/aeon_hip.h"
#include "jpeg.hpp" // jpeg_error: an error carrying its AEON_HIP_E* code

namespace aeon_hip {
namespace {

[[noreturn]] void png_bad(const std::string& m) { throw jpeg_error(AEON_HIP_EINVAL, "PNG: " + m); }

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};

struct PngHeader {
    int     w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
    int     samples = 0; // per pixel: 1 gray, 2 gray+alpha, 3 RGB, 4 RGBA, 1 palette index
    uint8_t pal[256][3]  = {};
    int     npal         = 0;
};

// Walk the chunks: IHDR, PLTE, the IDAT stream (concatenated); CRCs of critical chunks checked.
void parse(const uint8_t* d, size_t size, PngHeader& H, std::vector<uint8_t>* idat)
{
    if (size < 8 || std::memcmp(d, kSig, 8) != 0) png_bad("not a PNG file (bad signature)");
    size_t p        = 8;
    bool   got_ihdr = false, got_iend = false;
    while (p + 12 <= size) {
        const uint32_t len  = be32(d + p);
        const uint8_t* type = d + p + 4;
        if (len > size - p - 12) png_bad("truncated chunk");
        const uint8_t* data     = type + 4;
        const bool     critical = !(type[0] & 0x20);
        if (critical) {
            const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, len + 4);
            if (crc != be32(data + len)) png_bad(std::string("CRC error in ") + std::string((const char*)type, 4));
        }
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) png_bad("bad IHDR");
            H.w = (int)be32(data), H.h = (int)be32(data + 4), H.depth = data[8], H.ctype = data[9];
            H.interlace = data[12];
            if (H.w <= 0 || H.h <= 0 || H.w > (1 << 24) || H.h > (1 << 24)) png_bad("bad image size");
            if (data[10] != 0 || data[11] != 0 || H.interlace > 1) png_bad("unknown compression / filter / interlace method");
            switch (H.ctype) {
            case 0: H.samples = 1; break;
            case 2: H.samples = 3; break;
            case 3: H.samples = 1; break;
            case 4: H.samples = 2; break;
            case 6: H.samples = 4; break;
            default: png_bad("bad colour type");
            }
            const int d8 = H.depth;
            const bool ok = (H.ctype == 0 && (d8 == 1 || d8 == 2 || d8 == 4 || d8 == 8 || d8 == 16)) ||
                            (H.ctype == 3 && (d8 == 1 || d8 == 2 || d8 == 4 || d8 == 8)) ||
                            ((H.ctype == 2 || H.ctype == 4 || H.ctype == 6) && (d8 == 8 || d8 == 16));
            if (!ok) png_bad("bad bit depth for the colour type");
            got_ihdr = true;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (len % 3 || len == 0 || len > 768) png_bad("bad PLTE");
            H.npal = (int)len / 3;
            for (int i = 0; i < H.npal; i++) H.pal[i][0] = data[3 * i], H.pal[i][1] = data[3 * i + 1], H.pal[i][2] = data[3 * i + 2];
        } else if (!std::memcmp(type, "IDAT", 4)) {
            if (!got_ihdr) png_bad("IDAT before IHDR");
            if (idat) idat->insert(idat->end(), data, data + len);
            else return; // header only
        } else if (!std::memcmp(type, "IEND", 4)) {
            got_iend = true;
            break;
        }
        p += 12 + len;
    }
    if (!got_ihdr) png_bad("no IHDR");
    if (H.ctype == 3 && H.npal == 0) png_bad("palette image without PLTE");
    if (idat && !got_iend && idat->empty()) png_bad("no image data");
}

// Undo the row filters of a (sub-)image of w x h pixels whose filtered rows start at `in`.
void unfilter(uint8_t* in, int w, int h, int bpp_bits, std::vector<uint8_t>& out)
{
    const size_t rowb = ((size_t)w * bpp_bits + 7) / 8;
    const int    bpp  = std::max(1, bpp_bits / 8); // the filters' byte distance
    out.assign(rowb * h, 0);
    const uint8_t* prev = nullptr;
    for (int y = 0; y < h; y++) {
        const uint8_t  ft  = in[(rowb + 1) * y];
        const uint8_t* src = in + (rowb + 1) * y + 1;
        uint8_t*       dst = out.data() + rowb * y;
        switch (ft) {
        case 0: std::memcpy(dst, src, rowb); break;
        case 1:
            for (size_t i = 0; i < rowb; i++) dst[i] = (uint8_t)(src[i] + (i >= (size_t)bpp ? dst[i - bpp] : 0));
            break;
        case 2:
            for (size_t i = 0; i < rowb; i++) dst[i] = (uint8_t)(src[i] + (prev ? prev[i] : 0));
            break;
        case 3:
            for (size_t i = 0; i < rowb; i++) {
                const int a = i >= (size_t)bpp ? dst[i - bpp] : 0, b = prev ? prev[i] : 0;
                dst[i]      = (uint8_t)(src[i] + ((a + b) >> 1));
            }
            break;
        case 4:
            for (size_t i = 0; i < rowb; i++) {
                const int a = i >= (size_t)bpp ? dst[i - bpp] : 0, b = prev ? prev[i] : 0;
                const int c = (i >= (size_t)bpp && prev) ? prev[i - bpp] : 0;
                const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
                dst[i]      = (uint8_t)(src[i] + ((pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c)));
            }
            break;
        default: png_bad("bad filter type " + std::to_string(ft));
        }
        prev = dst;
    }
}

// Sample s (0-based) of a row of packed samples at `depth` bits, as an integer (16-bit big-endian)
inline uint32_t sample(const uint8_t* row, size_t s, int depth)
{
    switch (depth) {
    case 16: return (uint32_t)row[2 * s] << 8 | row[2 * s + 1];
    case 8: return row[s];
    default: {
        const size_t bit = s * depth;
        return (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1);
    }
    }
}

// libpng png_do_rgb_to_gray without gamma tables (png_set_rgb_to_gray(1, 0.299, 0.587)), as libpng
// 1.2 computes it at both depths: truncating >> 15.  (libpng 1.2.x is what the OpenCV 2.4.9 of
// aeon's README platform -- Ubuntu 16.04, libpng12 -- links; libpng >= 1.5.5 rounds the 16-bit case,
// + 16384 before the shift, which can differ by 1 in a 16-bit gray value.  Parity unpinned: no
// reference output holds a colour 16-bit PNG read as gray.)
constexpr uint32_t kRc = 29900u * 32768u / 100000u, kGc = 58700u * 32768u / 100000u, kBc = 32768u - kRc - kGc;
inline uint32_t rgb_to_gray(uint32_t r, uint32_t g, uint32_t b)
{
    return (r == g && r == b) ? r : (kRc * r + kGc * g + kBc * b) >> 15;
}

// Writes pixel (x, y) of the decoded picture in the requested form.
struct PngOut {
    int      mode;      // AEON_PNG_*
    int      out16;     // ANYDEPTH of a 16-bit file: uint16 samples
    uint8_t* dst;
    size_t   stride;
};

void png_emit_row(const PngHeader& H, const uint8_t* row, int npix, int x0, int dx, int y, const PngOut& O)
{
    uint8_t* d = O.dst + (size_t)y * O.stride;
    for (int i = 0; i < npix; i++) {
        const int x = x0 + i * dx;
        uint32_t  r, g, b; // in the file's depth, or 8 bits for palette / expanded gray
        const int depth = H.depth;
        bool      gray  = false;
        if (H.ctype == 3) {
            const uint32_t idx = sample(row, i, depth);
            if ((int)idx >= H.npal) png_bad("palette index out of range");
            r = H.pal[idx][0], g = H.pal[idx][1], b = H.pal[idx][2];
        } else if (H.ctype == 0 || H.ctype == 4) {
            uint32_t v = sample(row, (size_t)i * H.samples, depth);
            if (depth < 8) v = v * (depth == 1 ? 255 : depth == 2 ? 85 : 17);
            r = g = b = v, gray = true;
        } else {
            r = sample(row, (size_t)i * H.samples, depth), g = sample(row, (size_t)i * H.samples + 1, depth);
            b = sample(row, (size_t)i * H.samples + 2, depth);
        }
        const bool wide = depth == 16 && H.ctype != 3;
        if (O.mode == AEON_PNG_BGR8) {
            if (wide) r >>= 8, g >>= 8, b >>= 8; // png_set_strip_16: the high byte
            d[3 * x] = (uint8_t)b, d[3 * x + 1] = (uint8_t)g, d[3 * x + 2] = (uint8_t)r;
            continue;
        }
        uint32_t v = gray ? r : rgb_to_gray(r, g, b);
        if (O.out16) {
            const uint16_t w16 = (uint16_t)v;
            std::memcpy(d + 2 * (size_t)x, &w16, 2);
        } else {
            if (wide) v >>= 8;
            d[x] = (uint8_t)v;
        }
    }
}

} // namespace

void png_header(const void* data, size_t size, int* w, int* h, int* depth, int* ctype)
{
    PngHeader H;
    parse((const uint8_t*)data, size, H, nullptr);
    *w = H.w, *h = H.h, *depth = H.depth, *ctype = H.ctype;
}

void png_decode(const void* data, size_t size, int mode, void* dst, size_t stride, int* out_elem_bytes)
{
    PngHeader            H;
    std::vector<uint8_t> idat;
    parse((const uint8_t*)data, size, H, &idat);
    const int  bpp_bits = H.samples * H.depth;
    const bool out16    = mode == AEON_PNG_ANYDEPTH && H.depth == 16 && H.ctype != 3;
    if (out_elem_bytes) *out_elem_bytes = out16 ? 2 : 1;
    // inflated size: every (sub-)image's rows with their filter bytes
    static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
    const int passes = H.interlace ? 7 : 1;
    size_t    need   = 0;
    int       pw[7], ph[7];
    for (int k = 0; k < passes; k++) {
        pw[k] = H.interlace ? (H.w - ax0[k] + adx[k] - 1) / adx[k] : H.w;
        ph[k] = H.interlace ? (H.h - ay0[k] + ady[k] - 1) / ady[k] : H.h;
        if (pw[k] > 0 && ph[k] > 0) need += (((size_t)pw[k] * bpp_bits + 7) / 8 + 1) * ph[k];
    }
    std::vector<uint8_t> raw(need);
    z_stream             zs{};
    if (inflateInit(&zs) != Z_OK) png_bad("inflateInit failed");
    zs.next_in   = idat.data();
    zs.avail_in  = (uInt)idat.size();
    zs.next_out  = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    const size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR && zr != Z_OK) || got < need) png_bad("corrupt or truncated image data");
    PngOut               O{mode, out16 ? 1 : 0, (uint8_t*)dst, stride};
    std::vector<uint8_t> rows;
    size_t               off = 0;
    for (int k = 0; k < passes; k++) {
        if (pw[k] <= 0 || ph[k] <= 0) continue;
        unfilter(raw.data() + off, pw[k], ph[k], bpp_bits, rows);
        const size_t rowb = ((size_t)pw[k] * bpp_bits + 7) / 8;
        for (int y = 0; y < ph[k]; y++)
            png_emit_row(H, rows.data() + rowb * y, pw[k], H.interlace ? ax0[k] : 0, H.interlace ? adx[k] : 1,
                         H.interlace ? ay0[k] + y * ady[k] : y, O);
        off += (rowb + 1) * ph[k];
    }
}

} // namespace aeon_hip
