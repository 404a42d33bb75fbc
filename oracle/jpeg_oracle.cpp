// jpeg_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see aeon_oracle.h).
//
// CPU restatement of the JPEG decode behind aeon's image::extractor::extract
// (src/etl_image.cpp:83-99: cv::imdecode(..., CV_LOAD_IMAGE_COLOR / GRAYSCALE)).  OpenCV hands
// JPEG to libjpeg (the reference vendors neither): Ubuntu's libjpeg-turbo
// (libjpeg 6b/8 API) with its defaults -- JDCT_ISLOW, do_fancy_upsampling = TRUE -- and
// converts the RGB output to BGR (grayscale output for CV_LOAD_IMAGE_GRAYSCALE).  Restated here,
// as a plain dense decoder, from the published IJG algorithm:
//   * baseline / extended-sequential Huffman decoding, DRI restart intervals, interleaved and
//     non-interleaved scans (ITU T.81 F.2);
//   * jidctint.c jpeg_idct_islow (LL&M, CONST_BITS 13, PASS1_BITS 2) with the post-IDCT
//     range-limit table of jdmaster.c prepare_range_limit_table (x & 1023 wrap);
//   * jdsample.c: h2v1 / h2v2 / h1v2 fancy upsampling (triangle filters, context rows
//     replicated at the image edges as jdmainct.c does), box replication otherwise;
//   * jdcolor.c ycc_rgb_convert (SCALEBITS 16 fixed point tables); grayscale output = Y.
// Pinned by Pillow's libjpeg-turbo decodes of aeon's own JPEG fixtures (test/test_data/
// img_2112_70.jpg, flowers.jpg) and of JPEGs Pillow encodes (tests/golden/make_jpeg_fixtures.py).
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

const int kNatural[64 + 16] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
                               40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
                               29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
                               47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct Huff {
    bool     set = false;
    int      maxcode[18];
    int      valptr[17];
    int      mincode[17];
    uint8_t  vals[256];
};

struct Comp {
    int id, h, v, tq;
    int td = 0, ta = 0;
    int bw = 0, bh = 0;                 // blocks across / down (padded to the MCU grid)
    int dw = 0, dh = 0;                 // downsampled width / height
    std::vector<int16_t> coef;          // bw*bh blocks x 64, natural order
    int pred = 0;
};

struct Decoder {
    const uint8_t* p;
    const uint8_t* end;
    uint16_t       q[4][64];
    Huff           dc[4], ac[4];
    std::vector<Comp> comps;
    int            W = 0, H = 0, hmax = 1, vmax = 1, restart = 0, mcux = 0, mcuy = 0;
    bool           sof = false, adobe = false;
    int            adobe_transform = -1;
    // bit reader
    uint32_t bits = 0;
    int      nbits = 0;
    bool     hit_marker = false;

    [[noreturn]] void bad(const char* m) { throw std::runtime_error(std::string("jpeg: ") + m); }
    int u8()
    {
        if (p >= end) bad("truncated");
        return *p++;
    }
    int u16()
    {
        int a = u8();
        return (a << 8) | u8();
    }

    void build(Huff& t, const uint8_t* counts, const uint8_t* vals, int nvals)
    {
        std::memcpy(t.vals, vals, nvals);
        int code = 0, k = 0;
        for (int l = 1; l <= 16; l++) {
            t.valptr[l]  = k;
            t.mincode[l] = code;
            code += counts[l - 1];
            k += counts[l - 1];
            t.maxcode[l] = counts[l - 1] ? code - 1 : -1;
            code <<= 1;
        }
        t.maxcode[17] = 0x7fffffff;
        t.set         = true;
    }

    // entropy-coded segment bits (0xFF00 stuffing; a marker stops the supply and yields zeros)
    int bit()
    {
        if (nbits == 0) {
            int b = 0;
            if (!hit_marker) {
                if (p >= end) bad("truncated scan");
                b = *p;
                if (b == 0xFF) {
                    int nx = p + 1 < end ? p[1] : 0xD9;
                    if (nx == 0) p += 2;
                    else hit_marker = true, b = 0;
                } else {
                    p++;
                }
            }
            bits  = b;
            nbits = 8;
        }
        nbits--;
        return (bits >> nbits) & 1;
    }
    int receive(int s)
    {
        int v = 0;
        for (int i = 0; i < s; i++) v = (v << 1) | bit();
        return v;
    }
    static int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }
    int decode(const Huff& t)
    {
        if (!t.set) bad("undefined Huffman table");
        int code = bit(), l = 1;
        while (code > t.maxcode[l]) {
            code = (code << 1) | bit();
            if (++l > 16) bad("bad Huffman code");
        }
        return t.vals[t.valptr[l] + code - t.mincode[l]];
    }
    void block(Comp& c, int bx, int by)
    {
        int16_t* blk = &c.coef[((size_t)by * c.bw + bx) * 64];
        int      s   = decode(dc[c.td]);
        int      d   = s ? extend(receive(s), s) : 0;
        c.pred += d;
        blk[0] = (int16_t)c.pred;
        for (int k = 1; k < 64;) {
            int rs = decode(ac[c.ta]), r = rs >> 4;
            s = rs & 15;
            if (s) {
                k += r;
                blk[kNatural[k]] = (int16_t)extend(receive(s), s);
                k++;
            } else if (r == 15) {
                k += 16;
            } else {
                break;
            }
        }
    }
    void restart_marker()
    {
        nbits = 0;
        // skip to the RSTn marker
        while (p + 1 < end && !(p[0] == 0xFF && p[1] >= 0xD0 && p[1] <= 0xD7)) p++;
        if (p + 1 < end) p += 2;
        hit_marker = false;
        for (auto& c : comps) c.pred = 0;
    }
    void scan(const std::vector<int>& sc)
    {
        nbits = 0, hit_marker = false;
        for (auto& c : comps) c.pred = 0;
        int done = 0;
        if (sc.size() == 1) {
            Comp& c  = comps[sc[0]];
            int   nx = (c.dw + 7) / 8, ny = (c.dh + 7) / 8;
            for (int by = 0; by < ny; by++)
                for (int bx = 0; bx < nx; bx++) {
                    if (restart && done && done % restart == 0) restart_marker();
                    block(c, bx, by);
                    done++;
                }
        } else {
            for (int my = 0; my < mcuy; my++)
                for (int mx = 0; mx < mcux; mx++) {
                    if (restart && done && done % restart == 0) restart_marker();
                    for (int ci : sc) {
                        Comp& c = comps[ci];
                        for (int y = 0; y < c.v; y++)
                            for (int x = 0; x < c.h; x++) block(c, mx * c.h + x, my * c.v + y);
                    }
                    done++;
                }
        }
        // leave p at the next marker
        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) p++;
    }

    // progressive scans (ITU T.81 G.1.2; libjpeg jdphuff.c), coefficients in natural order
    bool progressive = false;
    int  eobrun      = 0;
    void refine(int16_t& c, int p1, int m1)
    {
        if (bit() && (c & p1) == 0) c = (int16_t)(c >= 0 ? c + p1 : c + m1);
    }
    void prog_block(Comp& c, int bx, int by, int Ss, int Se, int Ah, int Al)
    {
        int16_t*  blk = &c.coef[((size_t)by * c.bw + bx) * 64];
        const int p1 = 1 << Al, m1 = -p1;
        if (Ss == 0) { // DC (first: Huffman-coded difference; refine: one raw bit)
            if (Ah == 0) {
                int s = decode(dc[c.td]);
                c.pred += s ? extend(receive(s), s) : 0;
                blk[0] = (int16_t)(c.pred * p1);
            } else if (bit()) {
                blk[0] = (int16_t)(blk[0] | p1);
            }
            return;
        }
        int k = Ss;
        if (Ah == 0) { // AC first
            if (eobrun) {
                eobrun--;
                return;
            }
            while (k <= Se) {
                int rs = decode(ac[c.ta]), r = rs >> 4, s = rs & 15;
                if (s) {
                    k += r;
                    blk[kNatural[k]] = (int16_t)(extend(receive(s), s) * p1);
                } else if (r < 15) {
                    eobrun = (1 << r) - 1 + (r ? receive(r) : 0);
                    return;
                } else {
                    k += 15;
                }
                k++;
            }
            return;
        }
        if (!eobrun) { // AC refine
            while (k <= Se) {
                int rs = decode(ac[c.ta]), r = rs >> 4, s = rs & 15, v = 0;
                if (s) v = bit() ? p1 : m1;
                else if (r < 15) {
                    eobrun = (1 << r) + (r ? receive(r) : 0);
                    break;
                }
                while (k <= Se) {
                    int16_t& x = blk[kNatural[k]];
                    if (x) refine(x, p1, m1);
                    else if (r-- == 0) break;
                    k++;
                }
                if (v) blk[kNatural[k]] = (int16_t)v;
                k++;
            }
        }
        if (eobrun) {
            for (; k <= Se; k++)
                if (blk[kNatural[k]]) refine(blk[kNatural[k]], p1, m1);
            eobrun--;
        }
    }
    void prog_scan(const std::vector<int>& sc, int Ss, int Se, int Ah, int Al)
    {
        if ((Ss == 0 && Se != 0) || (Ss > 0 && (Se < Ss || Se > 63 || sc.size() != 1)) || Al > 13 ||
            (Ah && Al != Ah - 1))
            bad("bad progressive scan");
        nbits = 0, hit_marker = false, eobrun = 0;
        for (auto& c : comps) c.pred = 0;
        int done = 0;
        auto rst = [&] {
            if (restart && done && done % restart == 0) restart_marker(), eobrun = 0;
        };
        if (sc.size() == 1) {
            Comp& c = comps[sc[0]];
            for (int by = 0; by < (c.dh + 7) / 8; by++)
                for (int bx = 0; bx < (c.dw + 7) / 8; bx++, done++) rst(), prog_block(c, bx, by, Ss, Se, Ah, Al);
        } else {
            for (int my = 0; my < mcuy; my++)
                for (int mx = 0; mx < mcux; mx++, done++) {
                    rst();
                    for (int ci : sc)
                        for (int y = 0; y < comps[ci].v; y++)
                            for (int x = 0; x < comps[ci].h; x++)
                                prog_block(comps[ci], mx * comps[ci].h + x, my * comps[ci].v + y, Ss, Se, Ah, Al);
                }
        }
        while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) p++;
    }

    void parse()
    {
        if (u8() != 0xFF || u8() != 0xD8) bad("not a JPEG (no SOI)");
        for (;;) {
            int m = u8();
            if (m != 0xFF) bad("marker expected");
            while ((m = u8()) == 0xFF) {}
            if (m == 0xD9) break; // EOI
            if (m >= 0xD0 && m <= 0xD7) continue;
            int len = u16();
            const uint8_t* seg = p;
            if (len < 2 || p + len - 2 > end) bad("bad segment length");
            if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
                progressive = m == 0xC2;
                if (u8() != 8) bad("only 8-bit precision");
                H = u16(), W = u16();
                int n = u8();
                if (W <= 0 || H <= 0 || (n != 1 && n != 3)) bad("unsupported frame");
                comps.resize(n);
                for (auto& c : comps) {
                    c.id = u8();
                    int hv = u8();
                    c.h = hv >> 4, c.v = hv & 15, c.tq = u8();
                    if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) bad("bad component");
                    hmax = std::max(hmax, c.h), vmax = std::max(vmax, c.v);
                }
                mcux = (W + 8 * hmax - 1) / (8 * hmax);
                mcuy = (H + 8 * vmax - 1) / (8 * vmax);
                for (auto& c : comps) {
                    c.dw = (W * c.h + hmax - 1) / hmax;
                    c.dh = (H * c.v + vmax - 1) / vmax;
                    c.bw = mcux * c.h, c.bh = mcuy * c.v;
                    c.coef.assign((size_t)c.bw * c.bh * 64, 0);
                }
                sof = true;
            } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                bad("only Huffman baseline / extended sequential / progressive JPEGs");
            } else if (m == 0xC4) {
                while (p < seg + len - 2) {
                    int tc = u8(), th = tc & 15;
                    tc >>= 4;
                    if (th > 3 || tc > 1) bad("bad DHT");
                    uint8_t cnt[16];
                    int     tot = 0;
                    for (int i = 0; i < 16; i++) tot += cnt[i] = (uint8_t)u8();
                    if (tot > 256 || p + tot > end) bad("bad DHT");
                    build(tc ? ac[th] : dc[th], cnt, p, tot);
                    p += tot;
                }
            } else if (m == 0xDB) {
                while (p < seg + len - 2) {
                    int pq = u8(), tq = pq & 15;
                    pq >>= 4;
                    if (tq > 3) bad("bad DQT");
                    for (int i = 0; i < 64; i++) q[tq][kNatural[i]] = (uint16_t)(pq ? u16() : u8());
                }
            } else if (m == 0xDD) {
                restart = u16();
            } else if (m == 0xEE) {
                if (len >= 14 && std::memcmp(p, "Adobe", 5) == 0) adobe = true, adobe_transform = p[11];
                p = seg + len - 2;
            } else if (m == 0xDA) {
                if (!sof) bad("SOS before SOF");
                int              ns = u8();
                std::vector<int> sc;
                for (int i = 0; i < ns; i++) {
                    int cid = u8(), t = u8(), k = 0;
                    while (k < (int)comps.size() && comps[k].id != cid) k++;
                    if (k == (int)comps.size()) bad("bad scan component");
                    comps[k].td = t >> 4, comps[k].ta = t & 15;
                    sc.push_back(k);
                }
                const int Ss = u8(), Se = u8(), AhAl = u8();
                // jdinput.c per_scan_setup: JERR_BAD_MCU_SIZE past D_MAX_BLOCKS_IN_MCU (10) blocks per MCU
                if (ns > 1) {
                    int mb = 0;
                    for (int k : sc) mb += comps[k].h * comps[k].v;
                    if (mb > 10) bad("sampling factors too large for an interleaved scan");
                }
                p = seg + len - 2;
                if (progressive) prog_scan(sc, Ss, Se, AhAl >> 4, AhAl & 15);
                else scan(sc);
                continue;
            } else {
                p = seg + len - 2;
            }
            p = seg + len - 2;
        }
        if (!sof) bad("no frame");
        if (comps.size() == 3 && adobe && adobe_transform == 0) bad("RGB (Adobe transform 0) JPEGs are not supported");
    }
};

// jdmaster.c prepare_range_limit_table, post-IDCT part: clamp(x + 128) for |x| <= 511, wrap beyond
inline uint8_t idct_limit(int x)
{
    int i = x & 1023;
    if (i < 128) return (uint8_t)(i + 128);
    if (i < 512) return 255;
    if (i < 896) return 0;
    return (uint8_t)(i - 896);
}

// jidctint.c jpeg_idct_islow
void idct_islow(const int16_t* in, const uint16_t* qt, uint8_t* out, int stride)
{
    const long F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633, F1501 = 12299,
               F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
    int ws[64];
    for (int c = 0; c < 8; c++) {
        long z2 = (long)in[16 + c] * qt[16 + c], z3 = (long)in[48 + c] * qt[48 + c];
        long z1   = (z2 + z3) * F0541;
        long tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
        z2 = (long)in[c] * qt[c], z3 = (long)in[32 + c] * qt[32 + c];
        long tmp0 = (z2 + z3) * 8192, tmp1 = (z2 - z3) * 8192;
        long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
        tmp0 = (long)in[56 + c] * qt[56 + c], tmp1 = (long)in[40 + c] * qt[40 + c];
        tmp2 = (long)in[24 + c] * qt[24 + c], tmp3 = (long)in[8 + c] * qt[8 + c];
        z1 = tmp0 + tmp3, z2 = tmp1 + tmp2, z3 = tmp0 + tmp2;
        long z4 = tmp1 + tmp3, z5 = (z3 + z4) * F1175;
        tmp0 *= F0298, tmp1 *= F2053, tmp2 *= F3072, tmp3 *= F1501;
        z1 *= -F0899, z2 *= -F2562, z3 *= -F1961, z4 *= -F0390;
        z3 += z5, z4 += z5;
        tmp0 += z1 + z3, tmp1 += z2 + z4, tmp2 += z2 + z3, tmp3 += z1 + z4;
        auto d = [](long x) { return (int)((x + (1L << 10)) >> 11); };
        ws[c]      = d(t10 + tmp3), ws[56 + c] = d(t10 - tmp3);
        ws[8 + c]  = d(t11 + tmp2), ws[48 + c] = d(t11 - tmp2);
        ws[16 + c] = d(t12 + tmp1), ws[40 + c] = d(t12 - tmp1);
        ws[24 + c] = d(t13 + tmp0), ws[32 + c] = d(t13 - tmp0);
    }
    for (int r = 0; r < 8; r++) {
        const int* w  = ws + r * 8;
        long       z2 = w[2], z3 = w[6];
        long       z1 = (z2 + z3) * F0541;
        long tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
        long tmp0 = ((long)w[0] + w[4]) * 8192, tmp1 = ((long)w[0] - w[4]) * 8192;
        long t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
        tmp0 = w[7], tmp1 = w[5], tmp2 = w[3], tmp3 = w[1];
        z1 = tmp0 + tmp3, z2 = tmp1 + tmp2, z3 = tmp0 + tmp2;
        long z4 = tmp1 + tmp3, z5 = (z3 + z4) * F1175;
        tmp0 *= F0298, tmp1 *= F2053, tmp2 *= F3072, tmp3 *= F1501;
        z1 *= -F0899, z2 *= -F2562, z3 *= -F1961, z4 *= -F0390;
        z3 += z5, z4 += z5;
        tmp0 += z1 + z3, tmp1 += z2 + z4, tmp2 += z2 + z3, tmp3 += z1 + z4;
        auto d = [](long x) { return idct_limit((int)((x + (1L << 17)) >> 18)); };
        uint8_t* o = out + (size_t)r * stride;
        o[0] = d(t10 + tmp3), o[7] = d(t10 - tmp3), o[1] = d(t11 + tmp2), o[6] = d(t11 - tmp2);
        o[2] = d(t12 + tmp1), o[5] = d(t12 - tmp1), o[3] = d(t13 + tmp0), o[4] = d(t13 - tmp0);
    }
}

// jdsample.c: the component plane (dw x dh valid samples) upsampled to W x H
std::vector<uint8_t> upsample(const std::vector<uint8_t>& pl, int pw, const Comp& c, int hmax, int vmax, int W, int H)
{
    const int hf = hmax / c.h, vf = vmax / c.v;
    std::vector<uint8_t> out((size_t)W * H);
    const bool fancy = c.dw > 2;
    auto at = [&](int x, int y) { return (int)pl[(size_t)y * pw + x]; };
    if (hf == 1 && vf == 1) {
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)at(x, y);
        return out;
    }
    // one output row of h2v1 fancy from an input row accessor
    auto h2v1_row = [&](auto val, uint8_t* o) {
        const int        n = c.dw;
        std::vector<int> r(2 * n);
        r[0] = val(0);
        r[1] = (val(0) * 3 + val(1) + 2) >> 2;
        for (int i = 1; i < n - 1; i++) {
            r[2 * i]     = (val(i) * 3 + val(i - 1) + 1) >> 2;
            r[2 * i + 1] = (val(i) * 3 + val(i + 1) + 2) >> 2;
        }
        r[2 * n - 2] = (val(n - 1) * 3 + val(n - 2) + 1) >> 2;
        r[2 * n - 1] = val(n - 1);
        for (int x = 0; x < W; x++) o[x] = (uint8_t)r[x];
    };
    if (hf == 2 && vf == 1 && fancy) {
        for (int y = 0; y < H; y++) h2v1_row([&](int i) { return at(i, y); }, &out[(size_t)y * W]);
        return out;
    }
    if (hf == 1 && vf == 2 && fancy) { // libjpeg-turbo h1v2_fancy_upsample
        for (int y = 0; y < H; y++) {
            const int r = y / 2, v = y & 1;
            const int nb = v == 0 ? std::max(r - 1, 0) : std::min(r + 1, c.dh - 1);
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)((at(x, r) * 3 + at(x, nb) + (v ? 2 : 1)) >> 2);
        }
        return out;
    }
    if (hf == 2 && vf == 2 && fancy) { // h2v2_fancy_upsample
        const int n = c.dw;
        std::vector<int> cs(n);
        for (int y = 0; y < H; y++) {
            const int r = y / 2, v = y & 1;
            const int nb = v == 0 ? std::max(r - 1, 0) : std::min(r + 1, c.dh - 1);
            for (int i = 0; i < n; i++) cs[i] = at(i, r) * 3 + at(i, nb);
            std::vector<int> o(2 * n);
            o[0] = (cs[0] * 4 + 8) >> 4;
            o[1] = (cs[0] * 3 + cs[1] + 7) >> 4;
            for (int i = 1; i < n - 1; i++) {
                o[2 * i]     = (cs[i] * 3 + cs[i - 1] + 8) >> 4;
                o[2 * i + 1] = (cs[i] * 3 + cs[i + 1] + 7) >> 4;
            }
            o[2 * n - 2] = (cs[n - 1] * 3 + cs[n - 2] + 8) >> 4;
            o[2 * n - 1] = (cs[n - 1] * 4 + 7) >> 4;
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)o[x];
        }
        return out;
    }
    // box replication (h2v1_upsample / h2v2_upsample / int_upsample)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint8_t)at(x / hf, y / vf);
    return out;
}

inline uint8_t clamp255(int x) { return (uint8_t)(x < 0 ? 0 : (x > 255 ? 255 : x)); }

} // namespace

extern "C" {

thread_local std::string g_jpeg_err;

int orc_jpeg_info(const uint8_t* data, size_t size, int* w, int* h, int* ncomp)
{
    try {
        Decoder d;
        d.p = data, d.end = data + size;
        d.parse();
        *w = d.W, *h = d.H, *ncomp = (int)d.comps.size();
        return 0;
    } catch (const std::exception& e) {
        g_jpeg_err = e.what();
        return -1;
    }
}

// Decode to HWC: channels 3 -> BGR (gray JPEGs replicated), channels 1 -> grayscale (Y).
int orc_jpeg_decode(const uint8_t* data, size_t size, int channels, uint8_t* out)
{
    try {
        Decoder d;
        d.p = data, d.end = data + size;
        d.parse();
        const int W = d.W, H = d.H;
        std::vector<std::vector<uint8_t>> full;
        const int ncomp = channels == 1 ? 1 : (int)d.comps.size();
        for (int k = 0; k < ncomp; k++) {
            Comp&                c  = d.comps[k];
            const int            pw = c.bw * 8;
            std::vector<uint8_t> pl((size_t)pw * c.bh * 8);
            for (int by = 0; by < c.bh; by++)
                for (int bx = 0; bx < c.bw; bx++)
                    idct_islow(&c.coef[((size_t)by * c.bw + bx) * 64], d.q[c.tq], &pl[(size_t)by * 8 * pw + bx * 8], pw);
            full.push_back(upsample(pl, pw, c, d.hmax, d.vmax, W, H));
        }
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) {
                const size_t i = (size_t)y * W + x;
                if (channels == 1) {
                    out[i] = full[0][i];
                } else if (ncomp == 1) {
                    out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = full[0][i];
                } else {
                    const int Y = full[0][i], cb = full[1][i] - 128, cr = full[2][i] - 128;
                    const long r_cr = (91881L * cr + 32768) >> 16, b_cb = (116130L * cb + 32768) >> 16;
                    const long g    = (-22554L * cb + 32768 + -46802L * cr) >> 16;
                    out[3 * i + 2] = clamp255(Y + (int)r_cr);
                    out[3 * i + 1] = clamp255(Y + (int)g);
                    out[3 * i + 0] = clamp255(Y + (int)b_cb);
                }
            }
        return 0;
    } catch (const std::exception& e) {
        g_jpeg_err = e.what();
        return -1;
    }
}

const char* orc_jpeg_last_error(void) { return g_jpeg_err.c_str(); }

} // extern "C"
