// jpeg_host.cpp -- host half of the JPEG decode stage (see jpeg.hpp): header parsing, Huffman
// entropy decoding into the sparse coefficient stream on the decode pool, the per-call device
// layout, and the extern "C" entries aeon_jpeg_info / aeon_hip_decode_jpeg_batch.
//
// Follows libjpeg's Huffman decoders (ITU T.81 F.2 / G.1.2: DHT/DQT/DRI/SOF0-2/SOS, interleaved and
// non-interleaved scans, restart intervals, 0xFF00 stuffing; progressive files through spectral
// selection and successive approximation, jdphuff.c), which is what cv::imdecode runs under aeon's
// image::extractor::extract (src/etl_image.cpp:83-99).  Arithmetic-coded, lossless, 12-bit and
// 4-component (CMYK / Adobe RGB) files are refused with AEON_HIP_EUNSUPPORTED.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/aeon_hip.h"
#include "host.hpp"
#include "jpeg.hpp"
#include "jpeg_huff.hpp"

namespace aeon_hip {
hipError_t launch_jpeg(const JpegImage* imgs, const JpegChunk* chunks, int n_chunks, const JpegRows* rows, int n_rows,
                       int color_lds, hipStream_t stream);
int        jpeg_huff_stage_cap(int lanes);
hipError_t launch_jpeg_huff(const JpegHuffFile* files, int n_files, int lanes, int stage_bytes, int32_t* error,
                            hipStream_t stream);

namespace {

[[noreturn]] void bad(const std::string& m) { throw jpeg_error(AEON_HIP_EINVAL, "JPEG: " + m); }
[[noreturn]] void unsupported(const std::string& m) { throw jpeg_error(AEON_HIP_EUNSUPPORTED, "JPEG: " + m); }

const uint8_t kZigzagToNatural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
    6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31,
    39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

// AC fast table (kAcFastBits lookahead): a code of L <= kAcFastBits bits decodes in one lookup -- with its
// value when the value bits fit too (L + z <= kAcFastBits: kAcValue, value in bits 16-31), else its
// symbol (kAcSym: run in bits 5-8, size z in bits 16-19; the value bits follow with one get()).
// Entry: bits 0-4 bits consumed, 5-8 run, 9-11 kind (kAcValue, kAcEob, kAcZrl, kAcSym); 0 = a code
// longer than the lookahead (the general path).
constexpr int      kAcFastBits = 12;
constexpr uint32_t kAcValue = 1u << 9, kAcEob = 2u << 9, kAcZrl = 3u << 9, kAcSym = 4u << 9, kAcKind = 7u << 9;

// Canonical Huffman table with a 9-bit lookahead (libjpeg's jdhuff.c scheme).
struct Huffman {
    bool     set = false;
    uint16_t look[512]; // (length << 8) | symbol for codes of <= 9 bits, 0 otherwise
    int32_t  maxcode[18], valptr[17], mincode[17];
    uint8_t  vals[256];
    uint32_t fast[1 << kAcFastBits]; // AC tables: see kAcFastBits

    void build(const uint8_t* counts, const uint8_t* symbols, int n)
    {
        // validate the code space before any table entry is written (jdhuff.c
        // jpeg_make_d_derived_tbl: the code after the last one of length l must be < 2^l, so an
        // over-full length or an all-ones code is rejected)
        {
            int64_t code = 0;
            for (int l = 1; l <= 16; l++) {
                code += counts[l - 1];
                if (code >= ((int64_t)1 << l)) bad("bad Huffman table");
                code <<= 1;
            }
        }
        std::memcpy(vals, symbols, n);
        std::memset(look, 0, sizeof(look));
        int code = 0, k = 0;
        for (int l = 1; l <= 16; l++) {
            valptr[l]  = k;
            mincode[l] = code;
            for (int i = 0; i < counts[l - 1]; i++, k++, code++)
                if (l <= 9)
                    for (int f = 0; f < (1 << (9 - l)); f++) look[(code << (9 - l)) | f] = (uint16_t)((l << 8) | vals[k]);
            maxcode[l] = counts[l - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        // AC fast entries: every 10-bit window starting with a code of <= 10 bits
        std::memset(fast, 0, sizeof(fast));
        code = 0, k = 0;
        for (int l = 1; l <= kAcFastBits; l++) {
            for (int i = 0; i < counts[l - 1]; i++, k++, code++) {
                const int sym = vals[k], r = sym >> 4, z = sym & 15;
                for (int f = 0; f < (1 << (kAcFastBits - l)); f++) {
                    uint32_t e = 0;
                    if (sym == 0x00) e = kAcEob | (uint32_t)l;
                    else if (sym == 0xF0) e = kAcZrl | (uint32_t)l;
                    else if (z && l + z <= kAcFastBits) {
                        const int bits = (f >> (kAcFastBits - l - z)) & ((1 << z) - 1);
                        e = kAcValue | (uint32_t)(l + z) | ((uint32_t)r << 5) |
                            ((uint32_t)(uint16_t)(int16_t)extend(bits, z) << 16);
                    } else if (z) {
                        e = kAcSym | (uint32_t)l | ((uint32_t)r << 5) | ((uint32_t)z << 16);
                    }
                    fast[(code << (kAcFastBits - l)) | f] = e;
                }
            }
            code <<= 1;
        }
        set = true;
    }
};

// Entropy-coded segment reader: 64-bit buffer, 0xFF00 unstuffing; a marker ends the supply (zeros
// follow, as libjpeg's fill_bit_buffer does), running off the end of the file is an error.  fill()
// tops the buffer up to at least 57 bits once fewer than 32 are left, so one symbol (<= 16 bits)
// and its value bits (<= 16) follow without another check; eight bytes free of 0xFF go in with
// one load.  Every member that touches the
// state is inlined (nothing takes the reader's address), so a scan keeps it in registers.
struct Bits {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t       buf    = 0;
    int            n      = 0;
    bool           marker = false;

    [[gnu::always_inline]] void fill()
    {
        if (n >= 32) return; // enough for one symbol and its value bits
        if (!marker && end - p >= 8) {
            uint64_t w;
            std::memcpy(&w, p, 8);
            w                = __builtin_bswap64(w); // the next 8 bytes, first in the top byte
            const uint64_t x = ~w;                   // a 0xFF byte of w = a zero byte of x
            if (__builtin_expect(!((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull), 1)) {
                const int      k   = (64 - n) >> 3; // whole bytes that fit
                const uint64_t top = k == 8 ? w : (w >> (64 - 8 * k)) << (64 - 8 * k);
                buf |= top >> n;
                n += 8 * k;
                p += k;
                return;
            }
        }
        while (n <= 56) { // byte by byte: stuffing, markers, the end of the data
            uint64_t b = 0;
            if (!marker) {
                if (p >= end) bad("truncated scan data");
                b = *p;
                if (b == 0xFF) {
                    const int nx = p + 1 < end ? p[1] : 0xD9;
                    if (nx == 0) p += 2;
                    else marker = true, b = 0;
                } else {
                    p++;
                }
            }
            buf |= b << (56 - n);
            n += 8;
        }
    }
    // k in 1..16 bits; the caller has filled since the last symbol
    [[gnu::always_inline]] uint32_t get(int k)
    {
        const uint32_t v = (uint32_t)(buf >> (64 - k));
        buf <<= k;
        n -= k;
        return v;
    }
    // codes longer than 9 bits (the lookahead's miss): (symbol, length)
    [[gnu::noinline]] static uint32_t decode_long(const Huffman& t, uint64_t buf)
    {
        int l = 10;
        while (l <= 16 && (int32_t)(buf >> (64 - l)) > t.maxcode[l]) l++;
        if (l > 16) bad("corrupt Huffman code");
        const int code = (int)(buf >> (64 - l));
        return (uint32_t)t.vals[t.valptr[l] + code - t.mincode[l]] | ((uint32_t)l << 8);
    }
    [[gnu::always_inline]] int decode(const Huffman& t)
    {
        fill();
        uint32_t e = t.look[buf >> 55];
        if (!e) e = decode_long(t, buf);
        buf <<= e >> 8;
        n -= e >> 8;
        return e & 0xff;
    }
    // RSTn: drop buffered bits, skip to just past the marker; none left: zeros follow (libjpeg's
    // resync warns and decodes the missing intervals from no data)
    [[gnu::always_inline]] void restart()
    {
        buf = 0, n = 0, marker = false;
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) p++;
        if (p + 1 < end) p += 2;
        else marker = true;
    }
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0, td = 0, ta = 0;
    int bw = 0, bh = 0, dw = 0, dh = 0;
};

// Header of one file (and, once decoded, where its streams sit in the worker's arena).
struct Frame {
    int      W = 0, H = 0, ncomp = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool     progressive = false; // SOF2
    Comp     c[3];
    uint16_t q[4][64];
    bool     qset[4] = {false, false, false, false};
};

// The worker's growable output: block records then values per image (16-byte aligned pieces).
// A growable byte buffer: pageable, or pinned (the decode call's per-set arenas, which the H2D copies
// read directly).  Growing keeps the contents, as std::vector's resize does.
struct HostBuf {
    uint8_t* p      = nullptr;
    size_t   n      = 0;
    bool     pinned = false;
    HostBuf()       = default;
    HostBuf(const HostBuf&) = delete;
    HostBuf& operator=(const HostBuf&) = delete;
    HostBuf(HostBuf&& o) noexcept : p(o.p), n(o.n), pinned(o.pinned) { o.p = nullptr, o.n = 0; }
    ~HostBuf() { release(); }
    uint8_t* data() { return p; }
    size_t   size() const { return n; }
    void     release()
    {
        if (p) (void)(pinned ? hipHostFree(p) : (std::free(p), hipSuccess));
        p = nullptr, n = 0;
    }
    void resize(size_t m)
    {
        if (m <= n) return;
        uint8_t* q = nullptr;
        if (pinned) {
            if (hipHostMalloc((void**)&q, m, hipHostMallocDefault) != hipSuccess) q = nullptr;
        } else {
            q = (uint8_t*)std::malloc(m);
        }
        if (!q) throw jpeg_error(AEON_HIP_ERUNTIME, "JPEG arena allocation failed");
        if (n) std::memcpy(q, p, n);
        release();
        p = q, n = m;
    }
};

struct Arena {
    HostBuf              host; // staging the H2D reads (pinned in the decode call's sets)
    size_t               used = 0;
    std::vector<int16_t> coef; // progressive files: every block's 64 coefficients (zigzag order)
    std::vector<uint32_t> seg; // GPU-decoded files: segment starts while unstuffing
    uint8_t*             reserve(size_t bytes)
    {
        used = (used + 15) & ~(size_t)15;
        if (used + bytes > host.size()) host.resize(std::max(used + bytes, host.size() * 2));
        uint8_t* r = host.data() + used;
        used += bytes;
        return r;
    }
};

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

// Parse markers up to the frame header (SOF): size, components, sampling.
void parse_frame(const uint8_t* d, size_t size, Frame& f, const uint8_t** after)
{
    const uint8_t* p   = d;
    const uint8_t* end = d + size;
    if (size < 4 || p[0] != 0xFF || p[1] != 0xD8) bad("not a JPEG file (no SOI marker)");
    p += 2;
    for (;;) {
        while (p < end && *p != 0xFF) p++; // tolerate fill / garbage between segments
        while (p < end && *p == 0xFF) p++;
        if (p >= end) bad("no frame header");
        const int m = *p++;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (m == 0xD9) bad("no frame header");
        if (p + 2 > end) bad("truncated marker segment");
        const int len = be16(p);
        if (len < 2 || p + len > end) bad("truncated marker segment");
        const uint8_t* s = p + 2;
        if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
            f.progressive = m == 0xC2;
            if (len < 8) bad("bad frame header");
            if (s[0] != 8) unsupported("only 8-bit samples are supported");
            f.H = be16(s + 1), f.W = be16(s + 3), f.ncomp = s[5];
            if (f.W <= 0 || f.H <= 0) bad("bad image size");
            // (libjpeg would allocate whatever the header asks for; a bound keeps a corrupt header
            // from reserving gigabytes of coefficient staging)
            if ((int64_t)f.W * f.H > ((int64_t)1 << 28)) unsupported("images above 2^28 pixels");
            if (f.ncomp != 1 && f.ncomp != 3) unsupported("only 1- and 3-component images are supported");
            if (len < 8 + 3 * f.ncomp) bad("bad frame header");
            for (int k = 0; k < f.ncomp; k++) {
                Comp& c = f.c[k];
                c.id = s[6 + 3 * k], c.h = s[7 + 3 * k] >> 4, c.v = s[7 + 3 * k] & 15, c.tq = s[8 + 3 * k];
                if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) bad("bad component parameters");
                f.hmax = std::max(f.hmax, c.h), f.vmax = std::max(f.vmax, c.v);
            }
            for (int k = 0; k < f.ncomp; k++)
                if (f.hmax % f.c[k].h || f.vmax % f.c[k].v) unsupported("fractional sampling factors");
            f.mcux = (f.W + 8 * f.hmax - 1) / (8 * f.hmax);
            f.mcuy = (f.H + 8 * f.vmax - 1) / (8 * f.vmax);
            for (int k = 0; k < f.ncomp; k++) {
                Comp& c = f.c[k];
                c.dw = (f.W * c.h + f.hmax - 1) / f.hmax;
                c.dh = (f.H * c.v + f.vmax - 1) / f.vmax;
                c.bw = f.mcux * c.h, c.bh = f.mcuy * c.v;
            }
            *after = p + len;
            return;
        }
        if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)
            unsupported("only Huffman-coded baseline / extended-sequential / progressive JPEGs are supported (no "
                        "lossless, hierarchical or arithmetic coding)");
        p += len;
    }
}

// Decode one file: the frame's block records (per component, bh x bw, in the arena) and values.
// Returns the byte offsets in `a` of each component's records and of the values.
// One 8x8 block of a Huffman scan: its non-zero coefficients appended to vals (zigzag order) and
// their zigzag positions as the returned mask.  Inlined into the scan loops with the reader a
// local there, so the bit buffer stays in registers.
[[gnu::always_inline]] inline uint64_t decode_block(Bits& b, const Huffman& dct, const Huffman& act, int& pred,
                                                    int16_t* vals, uint32_t& nv)
{
    uint64_t  mask = 0;
    const int sdc  = b.decode(dct);
    if (sdc > 15) bad("corrupt DC coefficient");
    pred += sdc ? extend((int)b.get(sdc), sdc) : 0;
    const int16_t dcv = (int16_t)pred;
    if (dcv) mask |= 1, vals[nv++] = dcv;
    for (int k = 1; k < 64;) {
        b.fill();
        const uint32_t e    = act.fast[b.buf >> (64 - kAcFastBits)];
        const uint32_t kind = e & kAcKind;
        int            v;
        if (kind == kAcValue) { // code + value bits in one lookup
            const int used = e & 31;
            b.buf <<= used;
            b.n -= used;
            k += (e >> 5) & 15;
            v = (int16_t)(e >> 16);
        } else if (kind == kAcSym) { // the code's symbol; its value bits next (filled: <= 16 + 16 bits)
            const int used = e & 31, sz = (int)(e >> 16);
            b.buf <<= used;
            b.n -= used;
            k += (e >> 5) & 15;
            v = extend((int)b.get(sz), sz);
        } else if (e) { // EOB / ZRL
            b.buf <<= (e & 31);
            b.n -= (e & 31);
            if (kind == kAcEob) break;
            k += 16;
            continue;
        } else {
            const int rs = b.decode(act), r = rs >> 4, sz = rs & 15;
            if (!sz) {
                if (r != 15) break;
                k += 16;
                continue;
            }
            k += r;
            v = extend((int)b.get(sz), sz);
        }
        if (k < 63) {
            mask |= 1ull << k;
            vals[nv++] = (int16_t)v;
        } else if (mask >> 63 & 1) { // libjpeg's natural-order table clamps overruns to 63:
            vals[nv - 1] = (int16_t)v; // only that last value can repeat
        } else {
            mask |= 1ull << 63;
            vals[nv++] = (int16_t)v;
        }
        k++;
    }
    return mask;
}

// One scan of a progressive file (ITU T.81 G.1.2.1-2; libjpeg's jdphuff.c): DC first / refine
// (interleaved or not) and AC first / refine (one component) over the dense coefficients.
struct ProgScan {
    int Ss, Se, Ah, Al;
};

[[gnu::always_inline]] inline void refine_bit(Bits& b, int16_t& c, int p1, int m1)
{
    b.fill();
    if (b.get(1) && (c & p1) == 0) c = (int16_t)(c + (c >= 0 ? p1 : m1));
}

void decode_progressive_scan(Bits& br, const Frame& f, const int* sc, int ns, const ProgScan& S, const Huffman* dc,
                             const Huffman* ac, int restart, int16_t* const coef_of[3])
{
    const int p1 = 1 << S.Al, m1 = -p1;
    int       pred[3] = {0, 0, 0};
    int       eobrun  = 0;
    // block (bx, by) of scan component i
    auto dc_block = [&](int i, int16_t* blk) {
        const Comp& c = f.c[sc[i]];
        if (S.Ah == 0) {
            br.fill();
            const int t = br.decode(dc[c.td]);
            if (t > 15) bad("corrupt DC coefficient");
            br.fill();
            pred[i] += t ? extend((int)br.get(t), t) : 0;
            blk[0] = (int16_t)(pred[i] * (1 << S.Al));
        } else {
            br.fill();
            if (br.get(1)) blk[0] = (int16_t)(blk[0] | p1);
        }
    };
    auto ac_block = [&](int16_t* blk) {
        const Huffman& t = ac[f.c[sc[0]].ta];
        int            k = S.Ss;
        if (S.Ah == 0) { // AC first
            if (eobrun > 0) {
                eobrun--;
                return;
            }
            for (; k <= S.Se; k++) {
                const int rs = br.decode(t), r = rs >> 4, z = rs & 15;
                if (z) {
                    k += r;
                    br.fill();
                    // libjpeg's natural-order table clamps a corrupt run past 63 to 63
                    blk[std::min(k, 63)] = (int16_t)(extend((int)br.get(z), z) * (1 << S.Al));
                } else if (r == 15) {
                    k += 15;
                } else {
                    eobrun = (1 << r) - 1;
                    if (r) br.fill(), eobrun += (int)br.get(r);
                    break;
                }
            }
            return;
        }
        // AC refine
        if (eobrun == 0) {
            for (; k <= S.Se; k++) {
                const int rs = br.decode(t);
                int       r = rs >> 4, z = rs & 15, v = 0;
                if (z) { // (size 1 by construction; libjpeg only warns otherwise)
                    br.fill();
                    v = br.get(1) ? p1 : m1;
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) br.fill(), eobrun += (int)br.get(r);
                    break;
                }
                // past the coefficients already non-zero (refining each) and r zero ones
                for (; k <= S.Se; k++) {
                    int16_t& c = blk[k];
                    if (c != 0) refine_bit(br, c, p1, m1);
                    else if (--r < 0) break;
                }
                if (v) blk[std::min(k, 63)] = (int16_t)v;
            }
        }
        if (eobrun > 0) { // the band's remaining non-zero coefficients get their refinement bits
            for (; k <= S.Se; k++)
                if (blk[k] != 0) refine_bit(br, blk[k], p1, m1);
            eobrun--;
        }
    };
    int done = 0, left = restart;
    auto at_restart = [&]() {
        if (restart && done && left == 0) br.restart(), pred[0] = pred[1] = pred[2] = 0, eobrun = 0, left = restart;
    };
    if (ns == 1) { // non-interleaved: the component's own block grid
        const Comp& c  = f.c[sc[0]];
        const int   nx = (c.dw + 7) / 8, ny = (c.dh + 7) / 8;
        for (int by = 0; by < ny; by++)
            for (int bx = 0; bx < nx; bx++) {
                at_restart();
                int16_t* blk = coef_of[sc[0]] + ((size_t)by * c.bw + bx) * 64;
                if (S.Ss == 0) dc_block(0, blk);
                else ac_block(blk);
                done++, left--;
            }
        return;
    }
    for (int my = 0; my < f.mcuy; my++)
        for (int mx = 0; mx < f.mcux; mx++) {
            at_restart();
            for (int i = 0; i < ns; i++) {
                const Comp& c = f.c[sc[i]];
                for (int y = 0; y < c.v; y++)
                    for (int x = 0; x < c.h; x++)
                        dc_block(i, coef_of[sc[i]] + ((size_t)(my * c.v + y) * c.bw + mx * c.h + x) * 64);
            }
            done++, left--;
        }
}

void decode_file(const uint8_t* d, size_t size, Frame& f, Arena& a, size_t blk_off[3], size_t* val_off, bool luma_only)
{
    const uint8_t* p = nullptr;
    parse_frame(d, size, f, &p);
    const uint8_t* end = d + size;
    // re-walk the tables defined before the frame (DQT / DHT / DRI may precede SOF)
    Huffman dc[4], ac[4];
    int     restart = 0;
    bool    adobe_rgb = false;
    size_t  nblocks   = 0;
    for (int k = 0; k < f.ncomp; k++) nblocks += (size_t)f.c[k].bw * f.c[k].bh;
    // block records (zeroed: blocks a non-interleaved scan never codes stay empty), then values
    for (int k = 0; k < f.ncomp; k++) {
        uint8_t* b = a.reserve((size_t)f.c[k].bw * f.c[k].bh * sizeof(JpegBlock));
        std::memset(b, 0, (size_t)f.c[k].bw * f.c[k].bh * sizeof(JpegBlock));
        blk_off[k] = (size_t)(b - a.host.data());
    }
    // values: at most 64 per block
    uint8_t* vbase = a.reserve(nblocks * 64 * sizeof(int16_t));
    *val_off       = (size_t)(vbase - a.host.data());
    uint32_t nvals = 0;
    int16_t* coef_of[3] = {nullptr, nullptr, nullptr};
    if (f.progressive) { // scans refine a dense coefficient image; the sparse records come at the end
        a.coef.assign(nblocks * 64, 0);
        size_t o = 0;
        for (int k = 0; k < f.ncomp; k++) coef_of[k] = a.coef.data() + o, o += (size_t)f.c[k].bw * f.c[k].bh * 64;
    }
    auto table_segment = [&](int m, const uint8_t* s, int len) {
        const uint8_t* e = s + len - 2;
        if (m == 0xC4) {
            while (s < e) {
                const int tc = s[0] >> 4, th = s[0] & 15;
                if (tc > 1 || th > 3 || s + 17 > e) bad("bad Huffman table segment");
                int tot = 0;
                for (int i = 0; i < 16; i++) tot += s[1 + i];
                if (tot > 256 || s + 17 + tot > e) bad("bad Huffman table segment");
                (tc ? ac[th] : dc[th]).build(s + 1, s + 17, tot);
                s += 17 + tot;
            }
        } else if (m == 0xDB) {
            while (s < e) {
                const int pq = s[0] >> 4, tq = s[0] & 15;
                if (tq > 3 || pq > 1 || s + 1 + 64 * (pq + 1) > e) bad("bad quantisation table segment");
                for (int i = 0; i < 64; i++)
                    f.q[tq][kZigzagToNatural[i]] = pq ? be16(s + 1 + 2 * i) : s[1 + i];
                f.qset[tq] = true;
                s += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) {
            if (len < 4) bad("bad restart interval segment");
            restart = be16(s);
        } else if (m == 0xEE) {
            if (len >= 14 && std::memcmp(s, "Adobe", 5) == 0 && s[11] == 0) adobe_rgb = true;
        }
    };
    {
        // tables before SOF
        const uint8_t* q = d + 2;
        while (q < p) {
            while (q < p && *q != 0xFF) q++;
            while (q < p && *q == 0xFF) q++;
            if (q >= p) break;
            const int m = *q++;
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
            const int len = be16(q);
            if (m == 0xC0 || m == 0xC1 || m == 0xC2) break;
            table_segment(m, q + 2, len);
            q += len;
        }
    }
    bool any_scan = false;
    for (;;) {
        while (p < end && *p != 0xFF) p++;
        while (p < end && *p == 0xFF) p++;
        if (p >= end) {
            if (!any_scan) bad("no scan data");
            break; // missing EOI: tolerated, as libjpeg does
        }
        const int m = *p++;
        if (m == 0xD9) {
            if (!any_scan) bad("no scan data"); // (an image without a scan: libjpeg refuses it too)
            break;
        }
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (p + 2 > end) bad("truncated marker segment");
        const int len = be16(p);
        if (len < 2 || p + len > end) bad("truncated marker segment");
        if (m != 0xDA) {
            if ((m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)) bad("second frame header");
            table_segment(m, p + 2, len);
            p += len;
            continue;
        }
        // SOS
        if (len < 6) bad("bad scan header"); // (ns, the selectors and Ss/Se/Ah-Al need >= 4 bytes)
        const uint8_t* s  = p + 2;
        const int      ns = s[0];
        if (ns < 1 || ns > f.ncomp || len != 6 + 2 * ns) bad("bad scan header");
        int sc[3];
        for (int i = 0; i < ns; i++) {
            const int cid = s[1 + 2 * i], t = s[2 + 2 * i];
            int       k   = 0;
            while (k < f.ncomp && f.c[k].id != cid) k++;
            if (k == f.ncomp) bad("scan names an unknown component");
            f.c[k].td = t >> 4, f.c[k].ta = t & 15;
            if (f.c[k].td > 3 || f.c[k].ta > 3) bad("bad Huffman table selector");
            if (!f.qset[f.c[k].tq]) bad("component uses an undefined quantisation table");
            sc[i] = k;
        }
        // jdinput.c per_scan_setup: an interleaved scan's MCU holds at most D_MAX_BLOCKS_IN_MCU (10) blocks
        // (JERR_BAD_MCU_SIZE) -- cv::imdecode refuses such files, so they are refused here too
        if (ns > 1) {
            int mb = 0;
            for (int i = 0; i < ns; i++) mb += f.c[sc[i]].h * f.c[sc[i]].v;
            if (mb > 10) bad("sampling factors too large for an interleaved scan");
        }
        const ProgScan S{s[1 + 2 * ns], s[2 + 2 * ns], s[3 + 2 * ns] >> 4, s[3 + 2 * ns] & 15};
        if (f.progressive) {
            // jdphuff.c start_pass_phuff_decoder's checks
            const bool ok = (S.Ss == 0 ? S.Se == 0 : (S.Se >= S.Ss && S.Se <= 63 && ns == 1)) && S.Al <= 13 &&
                            (S.Ah == 0 || S.Al == S.Ah - 1);
            if (!ok) bad("bad progressive scan parameters");
            for (int i = 0; i < ns; i++) {
                const Comp& c = f.c[sc[i]];
                if ((S.Ss == 0 && S.Ah == 0 && !dc[c.td].set) || (S.Ss > 0 && !ac[c.ta].set))
                    bad("scan uses an undefined Huffman table");
            }
            p += len;
            any_scan = true;
            Bits br{p, end};
            decode_progressive_scan(br, f, sc, ns, S, dc, ac, restart, coef_of);
            p = br.p;
            while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) p++;
            continue;
        }
        for (int i = 0; i < ns; i++)
            if (!dc[f.c[sc[i]].td].set || !ac[f.c[sc[i]].ta].set) bad("scan uses an undefined Huffman table");
        if (S.Ss != 0 || S.Se != 63 || S.Ah != 0 || S.Al != 0)
            unsupported("progressive scan parameters in a sequential file");
        p += len;
        any_scan = true;
        Bits br{p, end};
        int16_t*  vals = (int16_t*)(a.host.data() + *val_off); // (no reallocation below: reserved)
        // a block coded twice (corrupt / duplicate scans) keeps the later values
        uint32_t nv   = nvals;
        int      done = 0, left = restart; // MCUs until the next restart marker
        if (ns == 1) {
            Comp&          c    = f.c[sc[0]];
            JpegBlock*     recs = (JpegBlock*)(a.host.data() + blk_off[sc[0]]);
            const Huffman& dct = dc[c.td];
            const Huffman& act = ac[c.ta];
            const int      nx = (c.dw + 7) / 8, ny = (c.dh + 7) / 8;
            int            pred = 0;
            for (int by = 0; by < ny; by++)
                for (int bx = 0; bx < nx; bx++) {
                    if (restart && done && left == 0) br.restart(), pred = 0, left = restart;
                    if (nv + 64 > nblocks * 64) bad("coefficient overflow (a block coded twice)");
                    JpegBlock& R = recs[(size_t)by * c.bw + bx];
                    R.val_off    = nv;
                    R.mask       = decode_block(br, dct, act, pred, vals, nv);
                    done++, left--;
                }
        } else {
            int pred[3] = {0, 0, 0};
            for (int my = 0; my < f.mcuy; my++)
                for (int mx = 0; mx < f.mcux; mx++) {
                    if (restart && done && left == 0) {
                        br.restart();
                        pred[0] = pred[1] = pred[2] = 0;
                        left = restart;
                    }
                    for (int i = 0; i < ns; i++) {
                        Comp&          c    = f.c[sc[i]];
                        JpegBlock*     recs = (JpegBlock*)(a.host.data() + blk_off[sc[i]]);
                        const Huffman& dct = dc[c.td];
                        const Huffman& act = ac[c.ta];
                        for (int y = 0; y < c.v; y++)
                            for (int x = 0; x < c.h; x++) {
                                if (nv + 64 > nblocks * 64) bad("coefficient overflow (a block coded twice)");
                                JpegBlock& R = recs[(size_t)(my * c.v + y) * c.bw + mx * c.h + x];
                                R.val_off    = nv;
                                R.mask       = decode_block(br, dct, act, pred[i], vals, nv);
                            }
                    }
                    done++, left--;
                }
        }
        nvals = nv;
        if (nvals > nblocks * 64) bad("coefficient overflow");
        // continue after the scan's data: the next marker that is not RSTn
        p = br.p;
        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) p++;
    }
    if (adobe_rgb && f.ncomp == 3) unsupported("RGB (Adobe transform 0) JPEGs");
    if (f.progressive) { // the dense coefficients as the sparse stream the kernels read
        int16_t* vals = (int16_t*)(a.host.data() + *val_off);
        for (int k = 0; k < f.ncomp; k++) {
            JpegBlock*     recs = (JpegBlock*)(a.host.data() + blk_off[k]);
            const int16_t* cb   = coef_of[k];
            for (size_t b = 0; b < (size_t)f.c[k].bw * f.c[k].bh; b++, cb += 64) {
                uint64_t mask = 0;
                recs[b].val_off = nvals;
                for (int z = 0; z < 64; z++)
                    if (cb[z]) mask |= 1ull << z, vals[nvals++] = cb[z];
                recs[b].mask = mask;
            }
        }
    }
    (void)luma_only;
    // give back the unused tail of the value reservation
    a.used = *val_off + (size_t)nvals * sizeof(int16_t);
}

// A file whose entropy decoding runs on the GPU (jpeg_huff.hip): where its pieces sit in the worker's
// arena and the scan's shape.
struct GpuScan {
    size_t   tabs = 0, segs = 0, sub_seg = 0, data = 0; // arena offsets
    int      nseg = 0, nsub = 0, restart = 0, n_mcu = 0, bpm = 0, mcux = 0, truncated = -1, sub_bits = 0, data_words = 0;
    bool     interleaved = false;
    uint64_t blk_tab[2] = {0, 0};
};

// jdhuff.c jpeg_make_d_derived_tbl's code-space check (as Huffman::build).
void check_code_space(const uint8_t* counts)
{
    int64_t code = 0;
    for (int l = 1; l <= 16; l++) {
        code += counts[l - 1];
        if (code >= ((int64_t)1 << l)) bad("bad Huffman table");
        code <<= 1;
    }
}

// The markers, tables and scan header of a file for the GPU entropy decoder, and its entropy-coded
// bytes unstuffed into the arena (segments split at RSTn when DRI is set; the data ends at the first
// other marker -- jdhuff.c's fill_bit_buffer: zeros follow a marker -- or with the file).  Returns false
// for the files the host decodes instead (decode_file): progressive (SOF2), a scan without every
// component (non-interleaved multi-scan), a second scan, more than kHuffMaxBpm blocks per MCU, data
// past 2^28 bytes.  Header errors throw as decode_file's do.
bool prepare_gpu(const uint8_t* d, size_t size, Frame& f, Arena& a, GpuScan& g, int lanes)
{
    const uint8_t* p = nullptr;
    parse_frame(d, size, f, &p);
    if (f.progressive) return false;
    const uint8_t* end   = d + size;
    const size_t   used0 = a.used;
    JpegHuffTab    dct[4], act[4];
    bool           dset[4] = {false, false, false, false}, aset[4] = {false, false, false, false};
    int            restart = 0;
    bool           adobe_rgb = false;
    auto segment = [&](int m, const uint8_t* s, int len) {
        const uint8_t* e = s + len - 2;
        if (m == 0xC4) {
            while (s < e) {
                const int tc = s[0] >> 4, th = s[0] & 15;
                if (tc > 1 || th > 3 || s + 17 > e) bad("bad Huffman table segment");
                int tot = 0;
                for (int i = 0; i < 16; i++) tot += s[1 + i];
                if (tot > 256 || s + 17 + tot > e) bad("bad Huffman table segment");
                check_code_space(s + 1);
                JpegHuffTab& t = tc ? act[th] : dct[th];
                std::memcpy(t.counts, s + 1, 16);
                std::memset(t.symbols, 0, sizeof(t.symbols));
                std::memcpy(t.symbols, s + 17, tot);
                (tc ? aset : dset)[th] = true;
                s += 17 + tot;
            }
        } else if (m == 0xDB) {
            while (s < e) {
                const int pq = s[0] >> 4, tq = s[0] & 15;
                if (tq > 3 || pq > 1 || s + 1 + 64 * (pq + 1) > e) bad("bad quantisation table segment");
                for (int i = 0; i < 64; i++) f.q[tq][kZigzagToNatural[i]] = pq ? be16(s + 1 + 2 * i) : s[1 + i];
                f.qset[tq] = true;
                s += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) {
            if (len < 4) bad("bad restart interval segment");
            restart = be16(s);
        } else if (m == 0xEE) {
            if (len >= 14 && std::memcmp(s, "Adobe", 5) == 0 && s[11] == 0) adobe_rgb = true;
        }
    };
    { // tables before SOF
        const uint8_t* q = d + 2;
        while (q < p) {
            while (q < p && *q != 0xFF) q++;
            while (q < p && *q == 0xFF) q++;
            if (q >= p) break;
            const int m = *q++;
            if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
            const int len = be16(q);
            if (m == 0xC0 || m == 0xC1 || m == 0xC2) break;
            segment(m, q + 2, len);
            q += len;
        }
    }
    // markers up to the scan
    int sc[3] = {0, 0, 0}, ns = 0;
    for (;;) {
        while (p < end && *p != 0xFF) p++;
        while (p < end && *p == 0xFF) p++;
        if (p >= end) bad("no scan data");
        const int m = *p++;
        if (m == 0xD9) bad("no scan data");
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (p + 2 > end) bad("truncated marker segment");
        const int len = be16(p);
        if (len < 2 || p + len > end) bad("truncated marker segment");
        if (m != 0xDA) {
            if ((m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)) bad("second frame header");
            segment(m, p + 2, len);
            p += len;
            continue;
        }
        if (len < 6) bad("bad scan header");
        const uint8_t* s = p + 2;
        ns               = s[0];
        if (ns < 1 || ns > f.ncomp || len != 6 + 2 * ns) bad("bad scan header");
        for (int i = 0; i < ns; i++) {
            const int cid = s[1 + 2 * i], t = s[2 + 2 * i];
            int       k   = 0;
            while (k < f.ncomp && f.c[k].id != cid) k++;
            if (k == f.ncomp) bad("scan names an unknown component");
            f.c[k].td = t >> 4, f.c[k].ta = t & 15;
            if (f.c[k].td > 3 || f.c[k].ta > 3) bad("bad Huffman table selector");
            if (!f.qset[f.c[k].tq]) bad("component uses an undefined quantisation table");
            sc[i] = k;
        }
        // jdinput.c per_scan_setup: an interleaved scan's MCU holds at most D_MAX_BLOCKS_IN_MCU (10) blocks
        // (JERR_BAD_MCU_SIZE) -- cv::imdecode refuses such files, so they are refused here too
        if (ns > 1) {
            int mb = 0;
            for (int i = 0; i < ns; i++) mb += f.c[sc[i]].h * f.c[sc[i]].v;
            if (mb > 10) bad("sampling factors too large for an interleaved scan");
        }
        if (ns != f.ncomp) return false; // components in separate scans: the host decoder
        for (int i = 0; i < ns; i++)
            if (!dset[f.c[sc[i]].td] || !aset[f.c[sc[i]].ta]) bad("scan uses an undefined Huffman table");
        if (s[1 + 2 * ns] != 0 || s[2 + 2 * ns] != 63 || s[3 + 2 * ns] != 0)
            unsupported("progressive scan parameters in a sequential file");
        p += len;
        break;
    }
    // the decoder's table slots: the scan's distinct DC tables in slots 0-1, its AC tables in 2-3 (a
    // scan naming more than two of either -- extended-sequential files may -- goes to the host decoder)
    int dslot[3] = {0, 0, 0}, aslot[3] = {0, 0, 0}, dids[2] = {-1, -1}, aids[2] = {-1, -1};
    for (int i = 0; i < ns; i++) {
        const int td = f.c[sc[i]].td, ta = f.c[sc[i]].ta;
        int       d = 0, q = 0;
        while (d < 2 && dids[d] >= 0 && dids[d] != td) d++;
        while (q < 2 && aids[q] >= 0 && aids[q] != ta) q++;
        if (d == 2 || q == 2) return false;
        dids[d] = td, aids[q] = ta, dslot[sc[i]] = d, aslot[sc[i]] = q;
    }
    // the scan's shape; each MCU block's byte: component | x << 2 | y << 4 | DC slot << 6 | AC slot - 2 << 7
    const bool inter = ns > 1;
    g.interleaved    = inter;
    g.bpm = 0, g.blk_tab[0] = g.blk_tab[1] = 0;
    if (inter) {
        for (int i = 0; i < ns; i++) {
            const Comp& c = f.c[sc[i]];
            for (int y = 0; y < c.v; y++)
                for (int x = 0; x < c.h; x++) {
                    if (g.bpm == kHuffMaxBpm) return false;
                    g.blk_tab[g.bpm >> 3] |= (uint64_t)(sc[i] | x << 2 | y << 4 | dslot[sc[i]] << 6 | aslot[sc[i]] << 7)
                                             << (8 * (g.bpm & 7));
                    g.bpm++;
                }
        }
        g.mcux = f.mcux, g.n_mcu = f.mcux * f.mcuy;
    } else {
        g.bpm = 1, g.blk_tab[0] = (uint64_t)(sc[0] | dslot[sc[0]] << 6 | aslot[sc[0]] << 7);
        g.mcux = (f.c[sc[0]].dw + 7) / 8, g.n_mcu = g.mcux * ((f.c[sc[0]].dh + 7) / 8);
    }
    g.restart = restart ? restart : g.n_mcu;
    const int nseg_need = (g.n_mcu + g.restart - 1) / g.restart;
    // unstuff the entropy-coded bytes into the arena (upper bound: what is left of the file)
    const size_t left = (size_t)(end - p);
    if (left >= ((size_t)1 << 28)) return false;
    g.data       = (size_t)(a.reserve(left + 16) - a.host.data());
    uint8_t* out = a.host.data() + g.data;
    size_t   o   = 0;
    auto&    seg = a.seg;
    seg.assign(1, 0);
    g.truncated = -1;
    for (;;) {
        const uint8_t* ff   = (const uint8_t*)std::memchr(p, 0xFF, (size_t)(end - p));
        const uint8_t* stop = ff ? ff : end;
        std::memcpy(out + o, p, (size_t)(stop - p));
        o += (size_t)(stop - p);
        if (!ff) { // the data runs into the end of the file
            g.truncated = (int)seg.size() - 1;
            p           = end;
            break;
        }
        const int nx = ff + 1 < end ? ff[1] : 0xD9;
        if (nx == 0) {
            out[o++] = 0xFF, p = ff + 2;
        } else if (restart && nx >= 0xD0 && nx <= 0xD7) {
            seg.push_back((uint32_t)o), p = ff + 2;
        } else if (restart && (int)seg.size() < nseg_need) {
            // another marker inside a restart interval: its data ends (zeros follow), and the next
            // interval starts after the next RSTn, wherever it is (decode_file's Bits::restart)
            const uint8_t* r = ff;
            while (r + 1 < end && !(r[0] == 0xFF && r[1] >= 0xD0 && r[1] <= 0xD7)) r++;
            if (r + 1 >= end) {
                p = ff;
                break;
            }
            seg.push_back((uint32_t)o), p = r + 2;
        } else {
            p = ff; // a marker ends the scan's data
            break;
        }
    }
    std::memset(out + o, 0, 16);
    a.used       = g.data + ((o + 16 + 3) & ~(size_t)3);
    g.data_words = (int)(((o + 16 + 3) & ~(size_t)3) / 4);
    // the markers after the scan: a second scan goes to the host decoder; Adobe APP14 as decode_file
    for (;;) {
        while (p < end && *p != 0xFF) p++;
        while (p < end && *p == 0xFF) p++;
        if (p >= end) break;
        const int m = *p++;
        if (m == 0xD9) break;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
        if (p + 2 > end) bad("truncated marker segment");
        const int len = be16(p);
        if (len < 2 || p + len > end) bad("truncated marker segment");
        if (m == 0xDA) {
            a.used = used0;
            return false;
        }
        if ((m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC)) bad("second frame header");
        if (m == 0xEE) segment(m, p + 2, len);
        p += len;
    }
    if (adobe_rgb && f.ncomp == 3) unsupported("RGB (Adobe transform 0) JPEGs");
    // segments: the ones past the scan's restart intervals are ignored, missing ones are empty;
    // subsequences: the data spread over the workgroup's lanes, within [kHuffSubMin, kHuffSubMax] bits
    // (longer when the segments' rounding up would give a lane more than one)
    std::vector<JpegHuffSeg> segs(nseg_need);
    for (int s = 0; s < nseg_need; s++) {
        const uint32_t b0 = s < (int)seg.size() ? seg[s] : (uint32_t)o;
        const uint32_t b1 = s + 1 < (int)seg.size() ? seg[s + 1] : (uint32_t)o;
        segs[s]           = {8 * b0, 8 * b1, 0, 0};
    }
    auto count = [&](int sub_bits) {
        int64_t c = 0;
        for (const JpegHuffSeg& S : segs) c += std::max<int64_t>(1, (S.end_bit - S.start_bit + sub_bits - 1) / sub_bits);
        return c;
    };
    const int64_t spread = ((int64_t)8 * o / std::max(lanes, 1) + 31) & ~(int64_t)31;
    g.sub_bits = (int)std::min<int64_t>(kHuffSubMax, std::max<int64_t>(kHuffSubMin, spread));
    while (g.sub_bits < kHuffSubMax && count(g.sub_bits) > lanes) g.sub_bits = std::min(kHuffSubMax, g.sub_bits + 32);
    int nsub = 0;
    for (JpegHuffSeg& S : segs) {
        S.first_sub = nsub;
        S.nsub      = std::max(1, (int)((S.end_bit - S.start_bit + g.sub_bits - 1) / g.sub_bits));
        nsub += S.nsub;
    }
    if (g.truncated >= nseg_need) g.truncated = -1; // (data of an ignored interval)
    g.nseg = nseg_need, g.nsub = nsub;
    // the scan's tables by slot (DC 0-1, AC 2-3; an unused slot has no codes), segments, subsequence -> segment
    g.tabs           = (size_t)(a.reserve(kJpegHuffSlots * sizeof(JpegHuffTab)) - a.host.data());
    JpegHuffTab* tab = (JpegHuffTab*)(a.host.data() + g.tabs);
    std::memset(tab, 0, kJpegHuffSlots * sizeof(JpegHuffTab));
    for (int d = 0; d < 2; d++)
        if (dids[d] >= 0) tab[d] = dct[dids[d]];
    for (int q = 0; q < 2; q++)
        if (aids[q] >= 0) tab[2 + q] = act[aids[q]];
    g.segs = (size_t)(a.reserve(segs.size() * sizeof(JpegHuffSeg)) - a.host.data());
    std::memcpy(a.host.data() + g.segs, segs.data(), segs.size() * sizeof(JpegHuffSeg));
    g.sub_seg   = (size_t)(a.reserve((size_t)nsub * sizeof(int32_t)) - a.host.data());
    int32_t* ss = (int32_t*)(a.host.data() + g.sub_seg);
    for (int s = 0; s < nseg_need; s++)
        for (int j = 0; j < segs[s].nsub; j++) *ss++ = s;
    return true;
}

} // namespace

// Per-context JPEG state: the decode pool, worker arenas, a two-deep ring of pinned staging +
// device buffers (a call reuses a set once the copies and kernels of the call before last are done).
struct JpegState {
    std::unique_ptr<thread_pool> own;
    thread_pool*                 pool = nullptr;
    struct Set {
        hipEvent_t done    = nullptr;
        hipEvent_t copied  = nullptr; // the set's H2D (on `copy`) is done: the call's kernels may start
        bool       pending = false;
        uint8_t*   pinned  = nullptr;
        size_t     pinned_cap = 0;
        uint8_t*   dev     = nullptr;
        size_t     dev_cap = 0;
        uint8_t*   planes  = nullptr;
        size_t     planes_cap = 0;
        uint8_t*   work    = nullptr; // GPU-decoded files: block records, dense coefficients, subsequence scratch
        size_t     work_cap = 0;
        std::vector<Arena> arenas;    // per pool worker, pinned: the H2D copies read them in place
    } sets[2];
    int         next = 0;
    hipStream_t copy = nullptr; // the H2D of a call's staging, so that it overlaps the previous call's
                                // kernels (AEON_HIP_JPEG_COPY_STREAM=0: on the call's stream)
    bool        use_copy = true;
    bool       gpu_huff = true; // false: every file through the host entropy decoder
    int        huff_lanes = kHuffLanes; // jpeg_huff workgroup size (AEON_HIP_JPEG_HUFF_LANES=256 / 1024: A/B)
    std::mutex mu;
};

namespace {

void grow_buf(uint8_t*& p, size_t& cap, size_t need, bool pinned)
{
    if (need <= cap) return;
    const size_t n = std::max(need, cap * 2);
    if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
    p = nullptr, cap = 0;
    hipError_t e = pinned ? hipHostMalloc((void**)&p, n, hipHostMallocDefault) : hipMalloc((void**)&p, n);
    if (e != hipSuccess) throw jpeg_error(AEON_HIP_ERUNTIME, std::string("JPEG staging allocation: ") + hipGetErrorString(e));
    cap = n;
}

void hip_ok(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw jpeg_error(AEON_HIP_ERUNTIME, std::string(what) + ": " + hipGetErrorString(e));
}

} // namespace

JpegState* jpeg_state_create(thread_pool* shared, bool gpu_huff)
{
    auto* s = new JpegState();
    s->gpu_huff = gpu_huff;
    if (const char* e = std::getenv("AEON_HIP_JPEG_COPY_STREAM")) s->use_copy = std::atoi(e) != 0;
    if (const char* e = std::getenv("AEON_HIP_JPEG_HUFF_LANES")) {
        const int l   = std::atoi(e);
        s->huff_lanes = l == 256 || l == 512 || l == 1024 ? l : kHuffLanes;
    }
    if (shared) {
        s->pool = shared;
    } else {
        std::vector<int> map = thread_affinity_map(""); // pinned like aeon's decode pool (AEON_CPU_LIST)
        if (const char* e = std::getenv("AEON_HIP_JPEG_THREADS")) map = affinity_for(map, std::max(1, std::atoi(e)));
        s->own.reset(new thread_pool(map));
        s->pool = s->own.get();
    }
    for (auto& st : s->sets) {
        st.arenas.resize(s->pool->size());
        for (auto& a : st.arenas) a.host.pinned = true;
    }
    return s;
}

void jpeg_state_destroy(JpegState* s)
{
    if (!s) return;
    for (auto& st : s->sets) {
        if (st.pending) (void)hipEventSynchronize(st.done);
        if (st.done) (void)hipEventDestroy(st.done);
        if (st.copied) (void)hipEventDestroy(st.copied);
        if (st.pinned) (void)hipHostFree(st.pinned);
        if (st.dev) (void)hipFree(st.dev);
        if (st.planes) (void)hipFree(st.planes);
        if (st.work) (void)hipFree(st.work);
    }
    if (s->copy) (void)hipStreamDestroy(s->copy);
    delete s;
}

// The decode call (aeon_hip_decode_jpeg_batch): on the pool, each file's headers, then either its
// entropy-coded bytes unstuffed for the GPU decoder (prepare_gpu) or the host entropy decoder's sparse
// stream (decode_file); all of it staged in one pinned buffer, one H2D, then jpeg_huff, the IDCT and
// the colour kernels on `stream`.  error: the context's device error word (corrupt entropy-coded data of
// a GPU-decoded file sets kJpegCorruptBit; aeon_hip_synchronize reports it).
// start / stop (may be null): events recorded around the GPU launches (kernel timing)
void jpeg_decode_batch(JpegState* S, int n, const void* const* data, const size_t* sizes, const aeon_img_desc* descs,
                       void* dst_base, int32_t* error, hipStream_t stream, hipEvent_t start, hipEvent_t stop)
{
    std::lock_guard<std::mutex> lock(S->mu);
    // (AEON_HIP_JPEG_PROFILE=1, development: host time per phase of each call on stderr)
    static const bool prof = std::getenv("AEON_HIP_JPEG_PROFILE") && std::atoi(std::getenv("AEON_HIP_JPEG_PROFILE"));
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    double tp[6] = {0};
    auto mark = [&](int k) {
        if (!prof) return;
        const auto t = clk::now();
        tp[k] = std::chrono::duration<double, std::micro>(t - t0).count();
        t0 = t;
    };
    // the call's set (pinned staging, device buffers, the workers' pinned arenas): reused once the
    // call that last used it is done with it
    JpegState::Set& st = S->sets[S->next];
    S->next ^= 1;
    if (!st.done) hip_ok(hipEventCreateWithFlags(&st.done, hipEventDisableTiming), "hipEventCreate");
    if (st.pending) hip_ok(hipEventSynchronize(st.done), "hipEventSynchronize");
    st.pending = false;
    mark(0);
    std::vector<Arena>& arenas = st.arenas;
    for (auto& a : arenas) a.used = 0;
    std::vector<Frame>   frames(n);
    std::vector<int>     owner(n);
    std::vector<size_t>  blk(3 * (size_t)n), val(n);
    std::vector<GpuScan> gs(n);
    std::vector<char>    on_gpu(n, 0);
    S->pool->run_indexed(n, [&](int i, int w) {
        try {
            if (!data[i] || !sizes[i]) bad("empty file");
            const aeon_img_desc& d = descs[i];
            if (d.channels != 1 && d.channels != 3) bad("decoded channels must be 1 or 3");
            const uint8_t* b = (const uint8_t*)data[i];
            if (S->gpu_huff && prepare_gpu(b, sizes[i], frames[i], arenas[w], gs[i], S->huff_lanes)) {
                on_gpu[i] = 1;
            } else {
                frames[i] = Frame();
                decode_file(b, sizes[i], frames[i], arenas[w], &blk[3 * (size_t)i], &val[i], d.channels == 1);
            }
            owner[i] = w;
            if (frames[i].W != d.width || frames[i].H != d.height)
                bad("decoded size " + std::to_string(frames[i].W) + "x" + std::to_string(frames[i].H) +
                    " does not match the record descriptor " + std::to_string(d.width) + "x" + std::to_string(d.height));
            if (d.stride < d.width * d.channels) bad("record descriptor stride too small");
        } catch (const jpeg_error& e) {
            throw jpeg_error(e.code, std::string(e.what()) + " (record " + std::to_string(i) + ")");
        }
    });
    mark(1);
    // device layout of the call: [images][GPU-decoded files][chunks][rows][arena 0][arena 1]...; the
    // work buffer (device only): [block records of the GPU-decoded files][their dense coefficients]
    // [their subsequence scratch]
    std::vector<JpegChunk> chunks;
    std::vector<JpegRows>  rows;
    // colour band height: kJpegRowsPerWg, or AEON_HIP_JPEG_BAND (tests: 1, 2, ... rows per workgroup
    // take the colour kernels' band-edge cases)
    int band_max = kJpegRowsPerWg;
    if (const char* e = std::getenv("AEON_HIP_JPEG_BAND"))
        if (std::atoi(e) >= 1) band_max = std::min(std::atoi(e), 64);
    size_t                 plane_bytes = 0;
    std::vector<size_t>    plane_off(3 * (size_t)n, 0);
    int                    color_lds = 0, n_gpu = 0;
    size_t                 rec_bytes = 0, coef_bytes = 0, sub_bytes = 0;
    std::vector<size_t>    wrec(3 * (size_t)n, 0), wcoef(3 * (size_t)n, 0), wsub(n, 0);
    for (int i = 0; i < n; i++) {
        const Frame& f  = frames[i];
        const int    nc = descs[i].channels == 1 ? 1 : f.ncomp; // grayscale output needs Y only
        if (on_gpu[i]) {
            n_gpu++;
            for (int k = 0; k < f.ncomp; k++) {
                const size_t nb = (size_t)f.c[k].bw * f.c[k].bh;
                wrec[3 * (size_t)i + k] = rec_bytes, rec_bytes += (nb * sizeof(JpegBlock) + 255) & ~(size_t)255;
                wcoef[3 * (size_t)i + k] = coef_bytes, coef_bytes += (nb * 64 * sizeof(int16_t) + 255) & ~(size_t)255;
            }
            wsub[i] = sub_bytes, sub_bytes += (size_t)gs[i].nsub * sizeof(JpegHuffSub);
        }
        for (int k = 0; k < nc; k++) {
            plane_off[3 * (size_t)i + k] = plane_bytes;
            plane_bytes += ((size_t)f.c[k].bw * 8 * f.c[k].bh * 8 + 255) & ~(size_t)255;
            const int nb = f.c[k].bw * f.c[k].bh;
            for (int b = 0; b < nb; b += kJpegIdctBlocks) chunks.push_back({i, k, b, std::min(kJpegIdctBlocks, nb - b)});
        }
        // colour bands: as many rows as the staged plane rows of the band fit the LDS (16 bytes more per
        // staged row: the 4:2:0 path's edge columns, jpeg_kernels.hip color_h2v2)
        int band = band_max, lds = 0;
        for (;; band /= 2) {
            lds = 0;
            for (int k = 0; k < nc; k++) {
                const int hf = f.hmax / f.c[k].h, vf = f.vmax / f.c[k].v;
                lds += jpeg_stage_rows(jpeg_upsample_mode(hf, vf, f.c[k].dw), vf, band) * (f.c[k].bw * 8 + 16);
            }
            if (lds <= kJpegColorLds || band == 1) break;
        }
        if (lds > kJpegColorLds) unsupported("image too wide for the colour pass's LDS rows");
        color_lds = std::max(color_lds, lds);
        for (int y = 0; y < f.H; y += band) rows.push_back({i, y, std::min(band, f.H - y), 0});
    }
    const size_t img_bytes = (size_t)n * sizeof(JpegImage);
    const size_t huf_off   = (img_bytes + 255) & ~(size_t)255;
    const size_t chk_off   = huf_off + (((size_t)n_gpu * sizeof(JpegHuffFile) + 255) & ~(size_t)255);
    const size_t row_off   = chk_off + ((chunks.size() * sizeof(JpegChunk) + 255) & ~(size_t)255);
    size_t       total     = row_off + ((rows.size() * sizeof(JpegRows) + 255) & ~(size_t)255);
    const size_t head = total; // descriptors and lists: staged in st.pinned; the arenas go up from their own
    std::vector<size_t> arena_off(arenas.size());
    for (size_t w = 0; w < arenas.size(); w++) {
        arena_off[w] = total;
        total += (arenas[w].used + 255) & ~(size_t)255;
    }
    mark(2);
    grow_buf(st.pinned, st.pinned_cap, head, true);
    grow_buf(st.dev, st.dev_cap, total, false);
    grow_buf(st.planes, st.planes_cap, std::max<size_t>(plane_bytes, 256), false);
    const size_t coef_off = rec_bytes, sub_off = rec_bytes + coef_bytes;
    if (n_gpu) grow_buf(st.work, st.work_cap, sub_off + sub_bytes, false);
    const uint64_t dev  = (uint64_t)st.dev, work = (uint64_t)st.work;
    JpegImage*     imgs = (JpegImage*)st.pinned;
    JpegHuffFile*  hf   = (JpegHuffFile*)(st.pinned + huf_off);
    int            huff_stage = 0; // LDS for the largest GPU-decoded file's data that fits the cap
    const int      stage_cap  = n_gpu ? jpeg_huff_stage_cap(S->huff_lanes) : 0;
    // The Huffman workgroups in order of entropy-coded size, largest first: dispatched in order, one
    // per CU per pass, workgroups i and i + 256 of a 512-file window share a CU, so each CU pairs a
    // long decode with a short one (in file order an alternating window put two large files on every
    // CU of half the XCDs).  Each descriptor carries its own outputs: the order changes nothing else.
    // A counting sort into 64 size classes gives each file its descriptor slot (hpos).
    std::vector<int> hpos(n, -1);
    {
        int64_t maxw = 1;
        for (int i = 0; i < n; i++)
            if (on_gpu[i]) maxw = std::max<int64_t>(maxw, gs[i].data_words);
        int  cnt[65] = {0};
        auto cls     = [&](int i) { return 63 - (int)((int64_t)gs[i].data_words * 63 / maxw); };
        for (int i = 0; i < n; i++)
            if (on_gpu[i]) cnt[cls(i) + 1]++;
        for (int c = 0; c < 64; c++) cnt[c + 1] += cnt[c];
        for (int i = 0; i < n; i++)
            if (on_gpu[i]) hpos[i] = cnt[cls(i)]++;
    }
    for (int i = 0; i < n; i++) {
        const Frame& f = frames[i];
        JpegImage&   J = imgs[i];
        std::memset(&J, 0, sizeof(J));
        const uint64_t base = dev + arena_off[owner[i]];
        for (int k = 0; k < f.ncomp; k++) {
            if (on_gpu[i]) {
                J.blocks[k] = work + wrec[3 * (size_t)i + k];
                J.dvals[k]  = work + coef_off + wcoef[3 * (size_t)i + k];
            } else {
                J.blocks[k] = base + blk[3 * (size_t)i + k];
            }
            J.planes[k] = (uint64_t)st.planes + plane_off[3 * (size_t)i + k];
            J.bw[k] = f.c[k].bw, J.bh[k] = f.c[k].bh, J.dw[k] = f.c[k].dw, J.dh[k] = f.c[k].dh;
            J.hs[k] = f.c[k].h, J.vs[k] = f.c[k].v;
            J.hf[k] = f.hmax / f.c[k].h, J.vf[k] = f.vmax / f.c[k].v;
            J.up[k] = jpeg_upsample_mode(J.hf[k], J.vf[k], f.c[k].dw);
            std::memcpy(J.q[k], f.q[f.c[k].tq], sizeof(J.q[k]));
            for (int z = 0; z < 64; z++) J.qz[k][z] = f.q[f.c[k].tq][kZigzagToNatural[z]];
        }
        J.values     = on_gpu[i] ? 0 : base + val[i];
        J.out        = (uint64_t)dst_base + descs[i].offset;
        J.W          = f.W, J.H = f.H, J.ncomp = f.ncomp, J.out_cn = descs[i].channels, J.out_stride = descs[i].stride;
        J.hmax       = f.hmax, J.vmax = f.vmax;
        if (!on_gpu[i]) continue;
        const GpuScan& g = gs[i];
        JpegHuffFile&  H = hf[hpos[i]];
        std::memset(&H, 0, sizeof(H));
        H.data    = base + g.data;
        H.segs    = base + g.segs;
        H.sub_seg = base + g.sub_seg;
        H.tabs    = base + g.tabs;
        H.subs    = work + sub_off + wsub[i];
        for (int k = 0; k < f.ncomp; k++) {
            H.blocks[k] = J.blocks[k], H.dvals[k] = J.dvals[k];
            H.bw[k] = f.c[k].bw;
            H.hs[k] = g.interleaved ? f.c[k].h : 1, H.vs[k] = g.interleaved ? f.c[k].v : 1;
        }
        H.blk_tab[0] = g.blk_tab[0], H.blk_tab[1] = g.blk_tab[1];
        H.nseg = g.nseg, H.nsub = g.nsub, H.restart = g.restart, H.n_mcu = g.n_mcu;
        H.bpm = g.bpm, H.mcux = g.mcux, H.ncomp = f.ncomp, H.truncated = g.truncated, H.sub_bits = g.sub_bits;
        H.data_words = g.data_words;
        if (g.data_words * 4 <= stage_cap) huff_stage = std::max(huff_stage, g.data_words * 4);
    }
    if (!chunks.empty()) std::memcpy(st.pinned + chk_off, chunks.data(), chunks.size() * sizeof(JpegChunk));
    if (!rows.empty()) std::memcpy(st.pinned + row_off, rows.data(), rows.size() * sizeof(JpegRows));
    mark(3);
    // (round 4 copied the arenas into st.pinned on the pool first: ~0.5 ms per 512 files)
    auto h2d = [&](hipStream_t on) {
        hip_ok(hipMemcpyAsync(st.dev, st.pinned, head, hipMemcpyHostToDevice, on), "hipMemcpyAsync");
        for (size_t w = 0; w < arenas.size(); w++)
            if (arenas[w].used)
                hip_ok(hipMemcpyAsync(st.dev + arena_off[w], arenas[w].host.data(), arenas[w].used, hipMemcpyHostToDevice, on),
                       "hipMemcpyAsync");
    };
    mark(4);
    if (S->use_copy) { // (the set's previous kernels are done: st.done above)
        if (!S->copy) hip_ok(hipStreamCreateWithFlags(&S->copy, hipStreamNonBlocking), "hipStreamCreate");
        if (!st.copied) hip_ok(hipEventCreateWithFlags(&st.copied, hipEventDisableTiming), "hipEventCreate");
        h2d(S->copy);
        hip_ok(hipEventRecord(st.copied, S->copy), "hipEventRecord");
        hip_ok(hipStreamWaitEvent(stream, st.copied, 0), "hipStreamWaitEvent");
    } else {
        h2d(stream);
    }
    if (n_gpu) hip_ok(hipMemsetAsync(st.work, 0, rec_bytes, stream), "hipMemsetAsync");
    if (start) hip_ok(hipEventRecord(start, stream), "hipEventRecord");
    if (n_gpu)
        hip_ok(launch_jpeg_huff((const JpegHuffFile*)(st.dev + huf_off), n_gpu, S->huff_lanes, huff_stage, error, stream),
               "JPEG Huffman kernel");
    hip_ok(launch_jpeg((const JpegImage*)st.dev, (const JpegChunk*)(st.dev + chk_off), (int)chunks.size(),
                       (const JpegRows*)(st.dev + row_off), (int)rows.size(), color_lds, stream),
           "JPEG kernels");
    if (stop) hip_ok(hipEventRecord(stop, stream), "hipEventRecord");
    hip_ok(hipEventRecord(st.done, stream), "hipEventRecord");
    st.pending = true;
    mark(5);
    if (prof)
        std::fprintf(stderr, "[jpeg stage] n=%d bytes=%zu us: set_wait %.0f pool %.0f layout %.0f fill %.0f h2d_setup %.0f enqueue %.0f\n",
                     n, total, tp[0], tp[1], tp[2], tp[3], tp[4], tp[5]);
}

// aeon_jpeg_info's body.
void jpeg_info(const void* data, size_t size, int* w, int* h, int* ncomp)
{
    Frame          f;
    const uint8_t* after = nullptr;
    parse_frame((const uint8_t*)data, size, f, &after);
    *w = f.W, *h = f.H, *ncomp = f.ncomp;
}

// aeon_jpeg_entropy_decode's body: the host half of the stage alone (headers, tables, every scan's
// Huffman decoding into the sparse block stream) on the calling thread -- no device needed.  The
// stream is summarised as its block and value counts and an FNV-1a hash of (mask, values) per block
// in component / raster order.
void jpeg_entropy_only(const void* data, size_t size, int* w, int* h, int* ncomp, int64_t* n_blocks,
                       int64_t* n_values, uint64_t* hash)
{
    Frame  f;
    Arena  a;
    size_t blk_off[3] = {0, 0, 0}, val_off = 0;
    decode_file((const uint8_t*)data, size, f, a, blk_off, &val_off, false);
    uint64_t  hv = 1469598103934665603ull;
    auto      mix = [&](uint64_t x) {
        for (int k = 0; k < 8; k++) hv = (hv ^ ((x >> (8 * k)) & 0xff)) * 1099511628211ull;
    };
    int64_t         nb = 0, nv = 0;
    const int16_t*  vals = (const int16_t*)(a.host.data() + val_off);
    for (int k = 0; k < f.ncomp; k++) {
        const JpegBlock* recs = (const JpegBlock*)(a.host.data() + blk_off[k]);
        for (size_t b = 0; b < (size_t)f.c[k].bw * f.c[k].bh; b++) {
            const int cnt = __builtin_popcountll(recs[b].mask);
            mix(recs[b].mask);
            for (int i = 0; i < cnt; i++) mix((uint64_t)(uint16_t)vals[recs[b].val_off + i]);
            nb++, nv += cnt;
        }
    }
    *w = f.W, *h = f.H, *ncomp = f.ncomp, *n_blocks = nb, *n_values = nv, *hash = hv;
}

// aeon_jpeg_host_stage's body: the batch decode's host work for one file on this thread -- headers
// and the unstuffed entropy-coded bytes for the GPU decoder, or the host entropy decoder's sparse
// stream -- and the bytes it stages for the H2D.
void jpeg_host_stage(const void* data, size_t size, int* gpu_entropy, int64_t* staged_bytes)
{
    Frame   f;
    Arena   a;
    GpuScan g;
    *gpu_entropy = prepare_gpu((const uint8_t*)data, size, f, a, g, kHuffLanes) ? 1 : 0;
    if (!*gpu_entropy) {
        size_t blk_off[3] = {0, 0, 0}, val_off = 0;
        f = Frame(), a.used = 0;
        decode_file((const uint8_t*)data, size, f, a, blk_off, &val_off, false);
    }
    *staged_bytes = (int64_t)a.used;
}

// The GPU entropy decoder's algorithm on this thread (host-only, for tests): prepare_gpu, then
// jpeg_huff's phases (jpeg_huff.hpp) one subsequence after another, the exclusive prefix serially --
// summarised as jpeg_entropy_only summarises the host decoder, so the two can be compared.  Returns 0
// when the file goes to the host decoder instead, 1 when decoded, -1 on corrupt entropy-coded data;
// *rounds: the Jacobi rounds until every start settled.
int jpeg_gpu_entropy_emulate(const void* data, size_t size, int lanes, int* w, int* h, int* ncomp, int64_t* n_blocks,
                             int64_t* n_values, uint64_t* hash, int* rounds)
{
    Frame   f;
    Arena   a;
    GpuScan g;
    if (!prepare_gpu((const uint8_t*)data, size, f, a, g, lanes)) return 0;
    std::vector<JpegBlock>   recs[3];
    std::vector<int16_t>     coef[3];
    std::vector<JpegHuffSub> subs(g.nsub);
    JpegHuffFile             F;
    std::memset(&F, 0, sizeof(F));
    uint8_t* base = a.host.data();
    F.data = (uint64_t)(base + g.data), F.segs = (uint64_t)(base + g.segs);
    F.sub_seg = (uint64_t)(base + g.sub_seg), F.tabs = (uint64_t)(base + g.tabs), F.subs = (uint64_t)subs.data();
    for (int k = 0; k < f.ncomp; k++) {
        const size_t nb = (size_t)f.c[k].bw * f.c[k].bh;
        recs[k].assign(nb, JpegBlock{0, 0, 0});
        coef[k].assign(nb * 64, 0);
        F.blocks[k] = (uint64_t)recs[k].data(), F.dvals[k] = (uint64_t)coef[k].data();
        F.bw[k] = f.c[k].bw, F.hs[k] = g.interleaved ? f.c[k].h : 1, F.vs[k] = g.interleaved ? f.c[k].v : 1;
    }
    F.blk_tab[0] = g.blk_tab[0], F.blk_tab[1] = g.blk_tab[1];
    F.nseg = g.nseg, F.nsub = g.nsub, F.restart = g.restart, F.n_mcu = g.n_mcu;
    F.bpm = g.bpm, F.mcux = g.mcux, F.ncomp = f.ncomp, F.truncated = g.truncated, F.sub_bits = g.sub_bits;
    F.data_words = g.data_words;
    std::unique_ptr<huff::Tables> T(new huff::Tables());
    huff::tables_codes(*T, F, 0, 1);
    huff::tables_fast(*T, F, 0, 1);
    huff::tables_long(*T, F, 0, 1);
    huff::pass_guess(*T, F, subs.data(), 0, 1);
    int r = 0;
    while (huff::pass_compare(F, subs.data(), 0, 1)) huff::pass_rewalk(*T, F, subs.data(), 0, 1), r++;
    int32_t acc[4] = {0, 0, 0, 0};
    for (auto& s : subs)
        for (int i = 0; i < 4; i++) s.ex[i] = acc[i], acc[i] += s.cnt[i];
    if (!huff::pass_write(*T, F, subs.data(), 0, 1)) return -1;
    uint64_t hv  = 1469598103934665603ull;
    auto     mix = [&](uint64_t x) {
        for (int b = 0; b < 8; b++) hv = (hv ^ ((x >> (8 * b)) & 0xff)) * 1099511628211ull;
    };
    int64_t nb = 0, nv = 0;
    for (int k = 0; k < f.ncomp; k++)
        for (size_t b = 0; b < recs[k].size(); b++) {
            const uint64_t m = recs[k][b].mask;
            mix(m);
            for (int z = 0; z < 64; z++)
                if (m >> z & 1) mix((uint64_t)(uint16_t)coef[k][b * 64 + z]), nv++;
            nb++;
        }
    *w = f.W, *h = f.H, *ncomp = f.ncomp, *n_blocks = nb, *n_values = nv, *hash = hv, *rounds = r;
    return 1;
}

} // namespace aeon_hip
