// jpeg_huff.hpp -- the GPU Huffman decoder's per-lane logic (jpeg_huff.hip), written once for the
// device and for the host: jpeg_huff runs its phases on a workgroup's lanes with barriers between
// them; jpeg_host.cpp's jpeg_gpu_entropy_emulate runs the same phases one subsequence after another
// (tests/sanitize/fuzz_driver.cpp compares it with the host entropy decoder on CPU).  See jpeg_huff.hip for the algorithm.
#pragma once
#include "jpeg.hpp"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define HUFF_FN __host__ __device__ __forceinline__
#else
#define HUFF_FN inline
#endif

// Device-memory pointers the walks read and write are address-space-1 (global) pointers on the device:
// generic (flat) accesses count on the LDS counter too, so every table lookup would wait for the bit
// reader's loads and the coefficient stores in flight.
#if defined(__HIP_DEVICE_COMPILE__)
#define HUFF_GLOBAL __attribute__((address_space(1)))
#else
#define HUFF_GLOBAL
#endif

namespace aeon_hip {
namespace huff {

template <typename T>
HUFF_FN HUFF_GLOBAL T* gmem(uint64_t a)
{
    return (HUFF_GLOBAL T*)a;
}

// Fast-table entry: bits 0-4 bits consumed, 5-8 AC run, 9-11 kind, 16-31 value (kValue) or value
// size (kSym).  0: no code of <= kHuffFastBits bits is a prefix (the long-code walk).
constexpr uint32_t kValue = 1u << 9, kEob = 2u << 9, kZrl = 3u << 9, kSym = 4u << 9, kKind = 7u << 9;
constexpr int      kTabs = kJpegHuffSlots; // the scan's DC tables (slots 0, 1), then its AC tables (2, 3)
constexpr int      kFast = 1 << kHuffFastBits;

constexpr int kLongSub = 16; // second-level tables per DHT table: codes of 11..16 bits by the 6 bits after
                             // their 10-bit prefix (canonical long codes share a few prefixes at the top)

struct Tables {
    uint32_t fast[kTabs][kFast];
    uint16_t longt[kTabs][kLongSub * 64]; // (length << 8) | symbol; 0: no code
    int32_t  long_first[kTabs];           // the first 10-bit prefix of a long code
    int32_t  maxcode[kTabs][17];          // largest code of each length (-1: none)
    int32_t  delta[kTabs][17];            // index of its first symbol - its first code
    uint8_t  vals[kTabs][256];
};

HUFF_FN int imin(int a, int b) { return a < b ? a : b; }
// v[comp] of three per-component values as arithmetic: a select chain over locals can become a
// stack lookup table (scratch memory) on the device
HUFF_FN int pick3(int comp, int a, int b, int c) { return a + (comp >= 1) * (b - a) + (comp >= 2) * (c - b); }
HUFF_FN uint64_t pick3(int comp, uint64_t a, uint64_t b, uint64_t c)
{
    return a + (uint64_t)(comp >= 1) * (b - a) + (uint64_t)(comp >= 2) * (c - b);
}
HUFF_FN int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

HUFF_FN void or_mask(HUFF_GLOBAL uint64_t* m, uint64_t v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    __hip_atomic_fetch_or(m, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *m |= v;
#endif
}

// Tables, part 1 (tables t0, t0 + dt, ...; symbols i0, i0 + di, ...): symbols, maxcode, delta.
HUFF_FN void tables_codes(Tables& T, const JpegHuffFile& F, int i0, int di)
{
    const HUFF_GLOBAL JpegHuffTab* tabs = gmem<const JpegHuffTab>(F.tabs);
    for (int i = i0; i < kTabs * 256; i += di) T.vals[i >> 8][i & 255] = tabs[i >> 8].symbols[i & 255];
    for (int t = i0; t < kTabs; t += di) {
        int code = 0, s = 0;
        for (int l = 1; l <= 16; l++) {
            const int n = tabs[t].counts[l - 1];
            T.delta[t][l]   = s - code;
            T.maxcode[t][l] = n ? code + n - 1 : -1;
            code = (code + n) << 1;
            s += n;
            if (l == kHuffFastBits) T.long_first[t] = code >> 1; // the 10-bit prefixes short codes leave
        }
    }
}

// Tables, part 3 (after part 1): the long-code subtables.
HUFF_FN void tables_long(Tables& T, const JpegHuffFile& F, int i0, int di)
{
    for (int i = i0; i < kTabs * kLongSub * 64; i += di) {
        const int t = i / (kLongSub * 64), r = i % (kLongSub * 64);
        const int prefix = T.long_first[t] + r / 64;
        uint16_t  e      = 0;
        if (prefix < kFast)
            for (int l = kHuffFastBits + 1; l <= 16; l++) {
                const int code = ((prefix << 6) | (r % 64)) >> (16 - l);
                if (code <= T.maxcode[t][l]) {
                    e = (uint16_t)((l << 8) | T.vals[t][T.delta[t][l] + code]);
                    break;
                }
            }
        T.longt[t][r] = e;
    }
}

// The entry of lookahead x (kHuffFastBits bits) of table t.
HUFF_FN uint32_t fast_entry(const Tables& T, int t, int x)
{
    for (int l = 1; l <= kHuffFastBits; l++) {
        const int code = x >> (kHuffFastBits - l);
        if (code > T.maxcode[t][l]) continue;
        const int sym = T.vals[t][T.delta[t][l] + code];
        if (t < 2) { // DC: the symbol is the difference's size
            if (sym <= 15 && l + sym <= kHuffFastBits) {
                const int bits = sym ? (x >> (kHuffFastBits - l - sym)) & ((1 << sym) - 1) : 0;
                const int v    = sym ? extend(bits, sym) : 0;
                return kValue | (uint32_t)(l + sym) | ((uint32_t)(uint16_t)(int16_t)v << 16);
            }
            return kSym | (uint32_t)l | ((uint32_t)sym << 16);
        }
        const int r = sym >> 4, z = sym & 15;
        if (!z) return (r == 15 ? kZrl : kEob) | (uint32_t)l; // (jdhuff.c: size 0, run < 15 ends the block)
        if (l + z <= kHuffFastBits) {
            const int bits = (x >> (kHuffFastBits - l - z)) & ((1 << z) - 1);
            return kValue | (uint32_t)(l + z) | ((uint32_t)r << 5) | ((uint32_t)(uint16_t)(int16_t)extend(bits, z) << 16);
        }
        return kSym | (uint32_t)l | ((uint32_t)r << 5) | ((uint32_t)z << 16);
    }
    return 0;
}

// Tables, part 2: the fast entries.
HUFF_FN void tables_fast(Tables& T, const JpegHuffFile& F, int i0, int di)
{
    for (int i = i0; i < kTabs * kFast; i += di) T.fast[i / kFast][i % kFast] = fast_entry(T, i / kFast, i % kFast);
}

// Bits of a segment: words at or past `end` read as zeros (libjpeg's fill after a marker).  64 bits
// in hand and the next word's load in flight: it is byte-swapped and masked only when a refill takes
// it, so its latency overlaps the codewords decoded meanwhile.
template <typename WP>
struct BitsT {
    WP                          w;    // the file's data as 32-bit words (device memory, or its LDS copy)
    int                         end;
    int                         last; // last word index holding segment bits (clamps the loads)
    uint64_t                    buf;  // next bits, first in bit 63
    int                         n;    // valid bits in buf
    int                         p;    // bit position of buf's bit 63
    uint32_t                    raw;  // word nw as loaded
    int                         nw;

    HUFF_FN uint32_t load(int i) const { return w[imin(i, last)]; }
    HUFF_FN uint32_t fix(uint32_t v, int i) const // big-endian, bits at or past `end` zeroed
    {
        v             = __builtin_bswap32(v);
        const int rem = end - i * 32;
        return rem >= 32 ? v : (rem <= 0 ? 0u : v & (0xffffffffu << (32 - rem)));
    }
    HUFF_FN void start(int pos)
    {
        const int i = pos >> 5, s = pos & 31;
        last = end > 0 ? (end - 1) >> 5 : 0;
        buf  = (((uint64_t)fix(load(i), i) << 32) | fix(load(i + 1), i + 1)) << s;
        n    = 64 - s;
        p    = pos;
        nw   = i + 2;
        raw  = load(nw);
    }
    // >= 32 valid bits: a code (<= 16) and its value bits (<= 15) without another check
    HUFF_FN void fill()
    {
        if (n < 32) {
            buf |= (uint64_t)fix(raw, nw) << (32 - n);
            n += 32;
            raw = load(++nw);
        }
    }
    // the same without a branch, for words in LDS: a word is read at every codeword (the same one
    // again when no refill was due)
    HUFF_FN void fill_always()
    {
        const bool need = n < 32;
        buf |= need ? (uint64_t)fix(raw, nw) << ((32 - n) & 63) : 0;
        n += need ? 32 : 0;
        nw += need ? 1 : 0;
        raw = load(nw);
    }
    HUFF_FN void skip(int l)
    {
        buf <<= l;
        n -= l;
        p += l;
    }
    HUFF_FN int get(int z) // 1..15 bits
    {
        const int v = (int)(buf >> (64 - z));
        skip(z);
        return v;
    }
};

using Bits = BitsT<const HUFF_GLOBAL uint32_t*>;

// Whether a walk's words are in device memory (a refill's load is kept a branch and loaded ahead)
// or in LDS (fill_always).
template <typename WP>
struct WordsInMemory {
    static constexpr bool value = false;
};
template <>
struct WordsInMemory<const HUFF_GLOBAL uint32_t*> {
    static constexpr bool value = true;
};

template <typename WP>
HUFF_FN BitsT<WP> bits_from(WP w, const JpegHuffSeg& S, int pos)
{
    BitsT<WP> b;
    b.w   = w;
    b.end = (int)S.end_bit;
    b.start(pos);
    return b;
}

HUFF_FN Bits bits_at(const JpegHuffFile& F, const JpegHuffSeg& S, int pos)
{
    return bits_from(gmem<const uint32_t>(F.data), S, pos);
}

HUFF_FN uint64_t pack_state(int p, int c, int k) { return (uint32_t)p | ((uint64_t)c << 32) | ((uint64_t)k << 40); }

// Where the blocks of a walk go (the final pass).
struct Out {
    int blk, blk_end; // current block (scan order), the segment's end
    int mx, my;       // MCU of the current block
    int pred0, pred1, pred2;
    int trunc; // reading past the segment's data is an error
};

// A code longer than the lookahead (fast entry 0) as a fast-table entry: the second-level table, or
// for prefixes beyond it the canonical maxcode walk.  *ok = false: no code of <= 16 bits (the entry
// then stands for a 1-bit code of symbol 0, a fixed continuation for a guessed start).
HUFF_FN uint32_t long_entry(const Tables& T, int t, uint64_t buf, bool& ok)
{
    const int sub = (int)(buf >> (64 - kHuffFastBits)) - T.long_first[t];
    int       l = 0, sym = 0;
    if (sub >= 0 && sub < kLongSub) {
        const int e = T.longt[t][sub * 64 + (int)((buf >> (64 - kHuffFastBits - 6)) & 63)];
        l = e >> 8, sym = e & 255;
    } else {
        for (int ll = kHuffFastBits + 1; ll <= 16; ll++) {
            const int code = (int)(buf >> (64 - ll));
            if (code <= T.maxcode[t][ll]) {
                l = ll, sym = T.vals[t][T.delta[t][ll] + code];
                break;
            }
        }
    }
    ok = l != 0;
    if (!ok) l = 1, sym = 0;
    if (t < 2) return kSym | (uint32_t)l | ((uint32_t)sym << 16);
    if (!(sym & 15)) return ((sym >> 4) == 15 ? kZrl : kEob) | (uint32_t)l; // (jdhuff.c: size 0, run < 15 ends the block)
    return kSym | (uint32_t)l | ((uint32_t)(sym >> 4) << 5) | ((uint32_t)(sym & 15) << 16);
}

// The MCU's block table in registers (F lives in device memory: a lane-dependent index into it would
// be a memory round trip at every block end).
struct BlkTab {
    uint64_t lo, hi;
    HUFF_FN int byte(int c) const { return (int)(((c < 8 ? lo : hi) >> (8 * (c & 7))) & 0xff); }
    HUFF_FN int comp(int c) const { return byte(c) & 3; }
    // the block's table slot: DC (slot 0 or 1) at k == 0, AC (2 or 3) after
    HUFF_FN int tab(int c, int k) const
    {
        const int by = byte(c);
        return k == 0 ? (by >> 6) & 1 : 2 + (by >> 7);
    }
};

// A sync walk from state (b.p, c, k) to the first codeword boundary at or past `stop`: blocks started
// and DC differences per component into cnt.  Written for a wave's lanes to stay together: a codeword
// is one fast-table lookup and a handful of selects; the only branches are the refill, a code longer
// than the lookahead and a DC difference whose bits exceed it.  AC value bits are skipped, not
// decoded.  (A guessed start can meet no-code bit patterns and DC sizes above 15: fixed continuations.)
template <typename B>
HUFF_FN void walk_sync(const Tables& T, const JpegHuffFile& F, B& b, int& c, int& k, int stop, int4& cnt)
{
    const BlkTab bt{F.blk_tab[0], F.blk_tab[1]};
    const int    bpm  = F.bpm;
    int          comp = bt.comp(c);
    while (b.p < stop) {
        if constexpr (WordsInMemory<decltype(b.w)>::value) b.fill();
        else b.fill_always();
        const int t = bt.tab(c, k);
        uint32_t  e = T.fast[t][(int)(b.buf >> (64 - kHuffFastBits))];
        if (!(e & kKind)) {
            bool ok;
            e = long_entry(T, t, b.buf, ok);
        }
        // the rest as selects: a wave's lanes take different kinds of codeword every time
        const uint32_t kind = e & kKind;
        const int      used = (int)(e & 31);
        const int      z    = kind == kSym ? imin((int)((e >> 16) & 0xff), 15) : 0;
        const int      zz   = z > 0 ? z : 1;
        const int      bits = (int)((b.buf << used) >> (64 - zz));
        const int      ext  = bits < (1 << (zz - 1)) ? bits - (1 << zz) + 1 : bits;
        const int      v    = kind == kValue ? (int)(int16_t)(e >> 16) : (z ? ext : 0); // (a DC difference)
        b.skip(used + z);
        const bool dc = k == 0;
        const int  vd = dc ? v : 0;
        cnt.x += dc ? 1 : 0;
        cnt.y += comp == 0 ? vd : 0;
        cnt.z += comp == 1 ? vd : 0;
        cnt.w += comp == 2 ? vd : 0;
        const int dk = kind == kEob ? 64 : (kind == kZrl ? 16 : (int)((e >> 5) & 15) + 1);
        k            = dc ? 1 : k + dk;
        const bool end = k >= 64;
        k              = end ? 0 : k;
        c              = end ? (c + 1 == bpm ? 0 : c + 1) : c;
        comp           = bt.comp(c);
    }
}

// The final walk from an exact state: every block's coefficients into its dense slots and its mask
// (plain store for a block this walk starts and ends, OR-ed where another walk holds part of it);
// up to the first codeword boundary at or past `stop`, or -- the segment's last subsequence -- until the
// segment's blocks are done.  Returns false on corrupt data: no code of <= 16 bits, a DC size above
// 15, bits past the end of a file whose data ends without a marker.
template <typename B>
HUFF_FN bool walk_write(const Tables& T, const JpegHuffFile& F, B& b, int& c, int& k, int stop, bool last, Out& o)
{
    const BlkTab          bt{F.blk_tab[0], F.blk_tab[1]};
    const int             bw0 = F.bw[0], bw1 = F.bw[1], bw2 = F.bw[2], hs0 = F.hs[0], hs1 = F.hs[1], hs2 = F.hs[2];
    const int             vs0 = F.vs[0], vs1 = F.vs[1], vs2 = F.vs[2], bpm = F.bpm, mcux = F.mcux;
    const uint64_t        dv0 = F.dvals[0], dv1 = F.dvals[1], dv2 = F.dvals[2];
    const uint64_t        bk0 = F.blocks[0], bk1 = F.blocks[1], bk2 = F.blocks[2];
    int                   comp = bt.comp(c);
    uint64_t              mask = 0;
    HUFF_GLOBAL int16_t*  coef = nullptr;
    HUFF_GLOBAL uint64_t* mrec = nullptr;
    bool                  own  = k == 0; // the current block started in this walk
    auto open = [&]() {                  // locate the current block in its component plane
        const int    by = bt.byte(c), x = (by >> 2) & 3, y = (by >> 4) & 3;
        const int    bw = pick3(comp, bw0, bw1, bw2), hs = pick3(comp, hs0, hs1, hs2), vs = pick3(comp, vs0, vs1, vs2);
        const size_t idx = (size_t)(o.my * vs + y) * bw + o.mx * hs + x;
        coef = gmem<int16_t>(pick3(comp, dv0, dv1, dv2)) + idx * 64;
        mrec = gmem<uint64_t>(pick3(comp, bk0, bk1, bk2)) + idx * 2;
    };
    if (o.blk < o.blk_end) open();
    while (o.blk < o.blk_end && (last || b.p < stop)) {
        b.fill();
        const int t = bt.tab(c, k);
        uint32_t  e = T.fast[t][(int)(b.buf >> (64 - kHuffFastBits))];
        if (!(e & kKind)) {
            bool ok;
            e = long_entry(T, t, b.buf, ok);
            if (!ok) return false;
        }
        const uint32_t kind = e & kKind;
        const int      used = (int)(e & 31);
        const int      z    = kind == kSym ? (int)((e >> 16) & 0xff) : 0;
        if (z > 15) return false; // (a DC size: the host decoder refuses it too)
        int v = kind == kValue ? (int)(int16_t)(e >> 16) : 0;
        if (z) v = extend((int)((b.buf << used) >> (64 - z)), z);
        b.skip(used + z);
        if (o.trunc && b.p > b.end) return false; // past the end of the file's data
        if (k == 0) { // DC difference
            const int pr = pick3(comp, o.pred0, o.pred1, o.pred2) + v;
            o.pred0 = comp == 0 ? pr : o.pred0;
            o.pred1 = comp == 1 ? pr : o.pred1;
            o.pred2 = comp == 2 ? pr : o.pred2;
            const int16_t dc = (int16_t)pr;
            if (dc) coef[0] = dc;
            mask = dc ? 1 : 0;
            k    = 1;
        } else if (kind == kEob || kind == kZrl) {
            k += kind == kEob ? 64 : 16;
        } else {
            k += (int)((e >> 5) & 15);
            const int zz = imin(k, 63); // jpeg_natural_order's extra entries clamp a run past 63 to 63
            mask |= 1ull << zz;
            coef[zz] = (int16_t)v;
            k++;
        }
        if (k >= 64) { // block done
            if (own) mrec[0] = mask;
            else if (mask) or_mask(mrec, mask);
            mask = 0, own = true;
            o.blk++;
            k = 0;
            if (++c == bpm) {
                c = 0;
                if (++o.mx == mcux) o.mx = 0, o.my++;
            }
            comp = bt.comp(c);
            if (o.blk < o.blk_end) open();
        }
    }
    if (k > 0 && mask) or_mask(mrec, mask); // a block split with the next subsequence
    return true;
}


template <typename S>
HUFF_FN void set_cnt(S& s, int4 v)
{
    s.cnt[0] = v.x, s.cnt[1] = v.y, s.cnt[2] = v.z, s.cnt[3] = v.w;
}
template <typename S>
HUFF_FN int4 get_ex(const S& s)
{
    return make_int4(s.ex[0], s.ex[1], s.ex[2], s.ex[3]);
}

// The phases below take the file's subsequence states `subs` (F.subs in device memory, or an LDS
// array when the file's subsequences fit the workgroup: on the device a pointer type of either
// address space).
// Where the guessed walk of the subsequence starting at bit p of segment S begins: kHuffLeadBits
// earlier (its guess at a block start re-synchronises over the lead-in), the segment's start (exact)
// when that is nearer.
HUFF_FN int guess_from(const JpegHuffSeg& S, int p) { return p - kHuffLeadBits <= (int)S.start_bit ? (int)S.start_bit : p - kHuffLeadBits; }

// The guessed walk: from guess_from (state block start), the state at the first codeword boundary at
// or past p is the subsequence's start st; when `ends` (not the segment's last subsequence), on to its
// end: en and the counts of its own bits.
template <typename B>
HUFF_FN void guess_walk(const Tables& T, const JpegHuffFile& F, const JpegHuffSeg& S, B b, int p, bool ends,
                        uint64_t& st, uint64_t& en, int4& cnt)
{
    int  c = 0, k = 0;
    int4 lead = make_int4(0, 0, 0, 0);
    walk_sync(T, F, b, c, k, p, lead);
    st  = pack_state(b.p, c, k);
    cnt = make_int4(0, 0, 0, 0);
    en  = 0;
    if (ends) {
        walk_sync(T, F, b, c, k, p + F.sub_bits, cnt);
        en = pack_state(b.p, c, k);
    }
}

// Phase 1: subsequences j0, j0 + dj, ... from their guessed starts.
template <typename SP>
HUFF_FN void pass_guess(const Tables& T, const JpegHuffFile& F, SP subs, int j0, int dj)
{
    const HUFF_GLOBAL JpegHuffSeg* segs = gmem<const JpegHuffSeg>(F.segs);
    const HUFF_GLOBAL int32_t*     sseg = gmem<const int32_t>(F.sub_seg);
    for (int j = j0; j < F.nsub; j += dj) {
        const JpegHuffSeg S = segs[sseg[j]];
        const int         i = j - S.first_sub, p = (int)S.start_bit + i * F.sub_bits;
        int4              cnt = make_int4(0, 0, 0, 0);
        uint64_t          st, en = 0;
        guess_walk(T, F, S, bits_at(F, S, guess_from(S, p)), p, i + 1 < S.nsub, st, en, cnt);
        subs[j].st = st;
        subs[j].en = en;
        set_cnt(subs[j], cnt);
    }
}

// Phase 2a: a start that differs from its predecessor's end takes it (ex[0]: walk again).  Returns
// whether any start changed.
template <typename SP>
HUFF_FN int pass_compare(const JpegHuffFile& F, SP subs, int j0, int dj)
{
    const HUFF_GLOBAL JpegHuffSeg* segs = gmem<const JpegHuffSeg>(F.segs);
    const HUFF_GLOBAL int32_t*     sseg = gmem<const int32_t>(F.sub_seg);
    int                any  = 0;
    for (int j = j0; j < F.nsub; j += dj) {
        const JpegHuffSeg S = segs[sseg[j]];
        int               dirty = 0;
        if (j > S.first_sub) {
            const uint64_t e = subs[j - 1].en;
            if (e != subs[j].st) subs[j].st = e, dirty = j + 1 < S.first_sub + S.nsub, any = 1;
        }
        subs[j].ex[0] = dirty;
    }
    return any;
}

// Phase 2b: walk the changed subsequences again from their new starts.
template <typename SP>
HUFF_FN void pass_rewalk(const Tables& T, const JpegHuffFile& F, SP subs, int j0, int dj)
{
    const HUFF_GLOBAL JpegHuffSeg* segs = gmem<const JpegHuffSeg>(F.segs);
    const HUFF_GLOBAL int32_t*     sseg = gmem<const int32_t>(F.sub_seg);
    for (int j = j0; j < F.nsub; j += dj) {
        if (!subs[j].ex[0]) continue;
        const JpegHuffSeg S  = segs[sseg[j]];
        const uint64_t    st = subs[j].st;
        const int         p = (int)(uint32_t)st, stop = (int)S.start_bit + (j - S.first_sub + 1) * F.sub_bits;
        int               c = (int)(st >> 32) & 0xff, k = (int)(st >> 40) & 0xff;
        int4              cnt = make_int4(0, 0, 0, 0);
        Bits              b   = bits_at(F, S, p);
        walk_sync(T, F, b, c, k, stop, cnt);
        subs[j].en = pack_state(b.p, c, k);
        set_cnt(subs[j], cnt);
    }
}

// Phase 4 (after the exclusive prefix of cnt into ex): the final decode.  Returns false if any of
// the walks met corrupt data.
template <typename SP>
HUFF_FN bool pass_write(const Tables& T, const JpegHuffFile& F, SP subs, int j0, int dj)
{
    const HUFF_GLOBAL JpegHuffSeg* segs = gmem<const JpegHuffSeg>(F.segs);
    const HUFF_GLOBAL int32_t*     sseg = gmem<const int32_t>(F.sub_seg);
    const int          per_seg = F.restart * F.bpm, total = F.n_mcu * F.bpm;
    bool               ok = true;
    for (int j = j0; j < F.nsub; j += dj) {
        const int         sg = sseg[j];
        const JpegHuffSeg S  = segs[sg];
        const int         i  = j - S.first_sub;
        const int4        e0 = get_ex(subs[S.first_sub]), e1 = get_ex(subs[j]);
        const uint64_t    st = subs[j].st;
        int               c = (int)(st >> 32) & 0xff, k = (int)(st >> 40) & 0xff;
        Out               o;
        o.blk     = sg * per_seg + (e1.x - e0.x) - (k > 0);
        o.blk_end = imin(sg * per_seg + per_seg, total);
        o.pred0 = e1.y - e0.y, o.pred1 = e1.z - e0.z, o.pred2 = e1.w - e0.w;
        o.trunc = F.truncated >= 0 && sg >= F.truncated;
        if (o.blk < sg * per_seg) continue; // (a continuation with no block before it cannot be exact)
        const int mcu = o.blk / F.bpm;
        o.mx = mcu % F.mcux, o.my = mcu / F.mcux;
        Bits b = bits_at(F, S, (int)(uint32_t)st);
        if (!walk_write(T, F, b, c, k, (int)S.start_bit + (i + 1) * F.sub_bits, i + 1 == S.nsub, o)) ok = false;
    }
    return ok;
}

} // namespace huff
} // namespace aeon_hip
