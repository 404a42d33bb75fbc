// jpeg_kernels.hip -- GPU half of the JPEG decode stage (see jpeg.hpp), bit-exact with libjpeg's
// defaults as cv::imdecode runs them under aeon's image::extractor::extract (etl_image.cpp:83-99).
//
// jpeg_idct: eight lanes per 8x8 block.  They gather the block's non-zero coefficients (the sparse
// stream of a host-decoded file, or the dense zigzag slots of a GPU-decoded one through an LDS
// scatter), dequantised, then run jidctint.c's jpeg_idct_islow (LL&M, CONST_BITS 13, PASS1_BITS 2;
// the post-IDCT range limit of jdmaster.c, x & 1023 wrap) -- integer multiply-adds only -- a column
// each, then a row each, and each lane writes its output row of the block into the component plane
// (one 8-byte store).
// jpeg_color: a workgroup per band of up to kJpegRowsPerWg output rows.  4:2:0 files with BGR output
// take color_h2v2 (8 columns of a row pair per lane, packed 16-bit upsampling); the others one lane
// per 4 output pixels of the band: each component sampled
// through jdsample.c's upsampler (h2v1 / h1v2 / h2v2 fancy triangle filters, context rows
// replicated at the edges as jdmainct.c does; box replication for the other ratios and for
// components narrower than 3 samples), then jdcolor.c ycc_rgb_convert (16-bit fixed point) and the
// BGR store of the decoded record into the augmentation stage's source arena.
#include <hip/hip_runtime.h>

#include "jpeg.hpp"

namespace aeon_hip {

// Device memory through address-space-1 pointers: generic (flat) loads and stores count on the LDS
// counter too, so the LDS transposes and upsampling reads would wait for them.
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
using gp = __attribute__((address_space(1))) T*;
#else
template <typename T>
using gp = T*; // (the host pass only parses the kernels)
#endif
template <typename T>
__device__ __forceinline__ gp<T> gaddr(uint64_t a)
{
    return (gp<T>)a;
}

__constant__ uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// range_limit[x & 1023] of jdmaster.c (prepare_range_limit_table, with the +CENTERJSAMPLE folded in):
// the low 10 bits as a signed value s, then clamp(s + 128, 0, 255) -- v_bfe_i32 + v_med3_i32
__device__ __forceinline__ uint32_t idct_limit(int x)
{
    const int s = __builtin_amdgcn_sbfe(x, 0, 10);
    return (uint32_t)min(max(s + 128, 0), 255);
}

// One 1-D LL&M pass on 8 values (in[0..7] at stride 1), results descaled by `shift`.
template <int SHIFT, bool FINAL>
__device__ __forceinline__ void llm8(const int* in, int* out)
{
    constexpr int F0298 = 2446, F0390 = 3196, F0541 = 4433, F0765 = 6270, F0899 = 7373, F1175 = 9633,
                  F1501 = 12299, F1847 = 15137, F1961 = 16069, F2053 = 16819, F2562 = 20995, F3072 = 25172;
    int z2 = in[2], z3 = in[6];
    int z1   = (z2 + z3) * F0541;
    int tmp2 = z1 + z3 * -F1847, tmp3 = z1 + z2 * F0765;
    int tmp0 = (in[0] + in[4]) * 8192, tmp1 = (in[0] - in[4]) * 8192;
    int t10 = tmp0 + tmp3, t13 = tmp0 - tmp3, t11 = tmp1 + tmp2, t12 = tmp1 - tmp2;
    tmp0 = in[7], tmp1 = in[5], tmp2 = in[3], tmp3 = in[1];
    z1 = tmp0 + tmp3, z2 = tmp1 + tmp2, z3 = tmp0 + tmp2;
    int z4 = tmp1 + tmp3, z5 = (z3 + z4) * F1175;
    tmp0 *= F0298, tmp1 *= F2053, tmp2 *= F3072, tmp3 *= F1501;
    z1 *= -F0899, z2 *= -F2562, z3 *= -F1961, z4 *= -F0390;
    z3 += z5, z4 += z5;
    tmp0 += z1 + z3, tmp1 += z2 + z4, tmp2 += z2 + z3, tmp3 += z1 + z4;
    constexpr int R = 1 << (SHIFT - 1);
    out[0] = (t10 + tmp3 + R) >> SHIFT, out[7] = (t10 - tmp3 + R) >> SHIFT;
    out[1] = (t11 + tmp2 + R) >> SHIFT, out[6] = (t11 - tmp2 + R) >> SHIFT;
    out[2] = (t12 + tmp1 + R) >> SHIFT, out[5] = (t12 - tmp1 + R) >> SHIFT;
    out[3] = (t13 + tmp0 + R) >> SHIFT, out[4] = (t13 - tmp0 + R) >> SHIFT;
}

// Natural index -> zigzag index (the inverse of kZz).
__constant__ uint8_t kZzInv[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                   3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                   10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                   21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// Eight lanes per block, the eight adjacent lanes of a wave, kJpegIdctUnroll blocks per lane group
// (group g takes blocks g, g + G, ... so concurrent lanes still write neighbouring blocks): first
// every block's descriptor, then every column gather, all loads in flight together.  A host-decoded
// file (sparse stream): lane j takes column j straight from the stream (coefficient at natural
// n = r*8 + j present iff its zigzag bit is set; its value index = the set bits below it).  A
// GPU-decoded file (dense zigzag slots): lane j takes zigzag slots 8j .. 8j + 7 of the block as one
// 16-byte load, dequantises them with the zigzag-ordered table (JpegImage.qz, one 16-byte load),
// zeroes those whose mask bit is clear (the slots are not cleared between calls) and scatters them
// to their natural positions in the group's LDS slot, from which it reads column j (block by
// block).  Then per block pass 1 in registers, a transpose through the same slot (wave barriers
// only) and pass 2 on row j.  Slot stride 66 dwords: lane (g, j) reads / writes column j of row r at
// bank (2g + 8r + j) % 64 -- conflict-free per wave.
constexpr int kSlot = 66;

__global__ __launch_bounds__(kJpegIdctLanes) void jpeg_idct(const JpegImage* __restrict__ imgs,
                                                            const JpegChunk* __restrict__ chunks)
{
    constexpr int G = kJpegIdctLanes / 8; // lane groups per workgroup
    constexpr int U = kJpegIdctUnroll;
    __shared__ int slot[G * kSlot];
    const JpegChunk  C  = chunks[blockIdx.x];
    const JpegImage& I  = imgs[C.img];
    const int        k  = C.comp;
    const int        g = threadIdx.x >> 3, j = threadIdx.x & 7;
    const gp<const JpegBlock> blocks = gaddr<const JpegBlock>(I.blocks[k]) + C.first;
    const gp<const int16_t>   vals   = gaddr<const int16_t>(I.values);
    const gp<const int16_t>   dense  = gaddr<const int16_t>(I.dvals[k]);
    JpegBlock        B[U];
#pragma unroll
    for (int u = 0; u < U; u++) B[u] = blocks[min(g + u * G, C.count - 1)];
    int* const s0 = slot + g * kSlot; // the group's block slot
    // pass 1 inputs: column j of every block, dequantised (jidctint.c DEQUANTIZE = coef * quantval)
    int col[U][8];
    if (dense) {
        uint4 c4[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            c4[u] = *(gp<const uint4>)(dense + (size_t)(C.first + min(g + u * G, C.count - 1)) * 64 + 8 * j);
        const uint4 q4 = *(gp<const uint4>)gaddr<const uint16_t>((uint64_t)&I.qz[k][8 * j]);
        int nat[8];
#pragma unroll
        for (int e = 0; e < 8; e++) nat[e] = kZz[8 * j + e];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t m8 = (uint32_t)(B[u].mask >> (8 * j)) & 0xffu;
            const uint32_t cw[4] = {c4[u].x, c4[u].y, c4[u].z, c4[u].w}, qw[4] = {q4.x, q4.y, q4.z, q4.w};
            if (u) { // the previous block's column reads are done
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
#pragma unroll
            for (int e = 0; e < 8; e++) {
                const int c = (int)(int16_t)(cw[e >> 1] >> (16 * (e & 1)));
                const int q = (int)((qw[e >> 1] >> (16 * (e & 1))) & 0xffff);
                s0[nat[e]] = ((m8 >> e) & 1) ? c * q : 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int r = 0; r < 8; r++) col[u][r] = s0[r * 8 + j];
        }
    } else {
        int qv[8];
#pragma unroll
        for (int r = 0; r < 8; r++) qv[r] = I.q[k][r * 8 + j];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int z = kZzInv[r * 8 + j];
                col[u][r]   = 0;
                if ((B[u].mask >> z) & 1)
                    col[u][r] = (int)vals[B[u].val_off + __builtin_popcountll(B[u].mask & ((1ull << z) - 1))] * qv[r];
            }
    }
    int* const  s   = s0;
    const int   bw  = I.bw[k];
    const float rbw = 1.0f / (float)bw;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const int bi = g + u * G;
        int       out[8], in[8];
        // pass 1: columns, descaled by CONST_BITS - PASS1_BITS
        llm8<11, false>(col[u], out);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier(); // the previous block's pass-2 reads are done
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int r = 0; r < 8; r++) s[r * 8 + j] = out[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // pass 2: row j, descaled by CONST_BITS + PASS1_BITS + 3, range limited; 8 bytes to the plane
#pragma unroll
        for (int c = 0; c < 8; c++) in[c] = s[j * 8 + c];
        llm8<18, true>(in, out);
        if (bi < C.count) {
            const int b  = C.first + bi;
            // b / bw through a float reciprocal: exact while bw < 512 ((b + 0.5) / bw stays 0.5 / bw from
            // an integer, far above the float error at these sizes)
            const int by = bw < 512 ? (int)(((float)b + 0.5f) * rbw) : b / bw, bx = b - by * bw;
            const gp<uint8_t> o = gaddr<uint8_t>(I.planes[k]) + (size_t)(by * 8 + j) * (bw * 8) + bx * 8;
            const uint32_t lo = idct_limit(out[0]) | idct_limit(out[1]) << 8 | idct_limit(out[2]) << 16 |
                                idct_limit(out[3]) << 24;
            const uint32_t hi = idct_limit(out[4]) | idct_limit(out[5]) << 8 | idct_limit(out[6]) << 16 |
                                idct_limit(out[7]) << 24;
            *(gp<uint2>)o = make_uint2(lo, hi);
        }
    }
}

// The geometry of one component as the colour pass uses it: its staged plane rows [lo, lo + n) in
// LDS (pitch pw), upsampler and sizes.
struct CompView {
    const uint8_t* P;
    int            lo, pw, dw, dh, up, hf, vf;
};

// The plane rows [lo, hi] of component k that output rows [y0, y1]'s upsampling reads (jdsample.c's
// context rows for the triangle filters, clamped at the image edges).
__device__ __forceinline__ void comp_rows(const JpegImage& I, int k, int y0, int y1, CompView& c, int& hi)
{
    c.pw = I.bw[k] * 8, c.dw = I.dw[k], c.dh = I.dh[k], c.up = I.up[k], c.hf = I.hf[k], c.vf = I.vf[k];
    if (c.up == UP_H1V2 || c.up == UP_H2V2) c.lo = max((y0 >> 1) - 1, 0), hi = min((y1 >> 1) + 1, c.dh - 1);
    else if (c.up == UP_BOX) c.lo = y0 / c.vf, hi = y1 / c.vf;
    else c.lo = y0, hi = y1;
}

// Sample (x, y) of the image from a component's plane through libjpeg's upsampler.
__device__ __forceinline__ int upsampled(const CompView& c, int x, int y)
{
    auto at = [&](int cx, int cy) { return (int)c.P[(cy - c.lo) * c.pw + cx]; };
    switch (c.up) {
    case UP_FULL: return at(x, y);
    case UP_H2V1: { // h2v1_fancy_upsample
        const int i = x >> 1;
        if ((x & 1) == 0) return i == 0 ? at(0, y) : (at(i, y) * 3 + at(i - 1, y) + 1) >> 2;
        return i == c.dw - 1 ? at(i, y) : (at(i, y) * 3 + at(i + 1, y) + 2) >> 2;
    }
    case UP_H1V2: { // h1v2_fancy_upsample (libjpeg-turbo)
        const int r = y >> 1, v = y & 1;
        const int nb = v == 0 ? max(r - 1, 0) : min(r + 1, c.dh - 1);
        return (at(x, r) * 3 + at(x, nb) + (v ? 2 : 1)) >> 2;
    }
    case UP_H2V2: { // h2v2_fancy_upsample
        const int r = y >> 1, v = y & 1;
        const int nb = v == 0 ? max(r - 1, 0) : min(r + 1, c.dh - 1);
        const int i  = x >> 1;
        auto cs = [&](int ci) { return at(ci, r) * 3 + at(ci, nb); };
        const int t = cs(i);
        if ((x & 1) == 0) return i == 0 ? (t * 4 + 8) >> 4 : (t * 3 + cs(i - 1) + 8) >> 4;
        return i == c.dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + cs(i + 1) + 7) >> 4;
    }
    default: return at(x / c.hf, y / c.vf); // h2v1_upsample / h2v2_upsample / int_upsample
    }
}

// Output rows [y0, y0 + rows) of image I from its staged component rows cv: one lane per 4 consecutive
// pixels -- one dword (gray) or three dwords (BGR) when the group is whole and 4-byte aligned,
// bytewise otherwise.
__device__ __forceinline__ void color_rows(const JpegImage& I, const CompView* cv, int y0, int nrows)
{
    const int W = I.W, cn = I.out_cn, nc = cn == 1 ? 1 : I.ncomp;
    const gp<uint8_t> out = gaddr<uint8_t>(I.out);
    const int         stride = I.out_stride;
    const int groups = (W + 3) >> 2;
    for (int q = threadIdx.x; q < groups * nrows; q += blockDim.x) {
        const int y = y0 + q / groups, x0 = (q % groups) * 4;
        uint32_t  p[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int x = min(x0 + e, W - 1);
            const int Y = upsampled(cv[0], x, y);
            if (nc == 1) {
                p[e] = cn == 1 ? (uint32_t)Y : (uint32_t)Y * 0x010101u;
            } else {
                const int cb = upsampled(cv[1], x, y) - 128, cr = upsampled(cv[2], x, y) - 128;
                const int r  = Y + ((91881 * cr + 32768) >> 16);
                const int g  = Y + ((-22554 * cb + 32768 + -46802 * cr) >> 16);
                const int bl = Y + ((116130 * cb + 32768) >> 16);
                p[e] = (uint32_t)min(max(bl, 0), 255) | (uint32_t)min(max(g, 0), 255) << 8 |
                       (uint32_t)min(max(r, 0), 255) << 16;
            }
        }
        const gp<uint8_t> o = out + (size_t)y * stride + (size_t)x0 * cn;
        if (x0 + 3 < W && ((uintptr_t)o & 3) == 0) {
            if (cn == 1) {
                *(gp<uint32_t>)o = p[0] | p[1] << 8 | p[2] << 16 | p[3] << 24;
            } else {
                const gp<uint32_t> d = (gp<uint32_t>)o;
                d[0] = p[0] | p[1] << 24;
                d[1] = p[1] >> 8 | p[2] << 16;
                d[2] = p[2] >> 16 | p[3] << 8;
            }
        } else {
            for (int e = 0; e < 4 && x0 + e < W; e++)
                for (int c = 0; c < cn; c++) o[e * cn + c] = (uint8_t)(p[e] >> (8 * c));
        }
    }
}

// ---- 4:2:0 BGR fast path (luma full, both chroma h2v2_fancy_upsample) --------------------------
// A lane owns 8 output columns x0 = 8q.. of an output row pair (2r, 2r + 1), which share chroma row
// r: per chroma it takes columns i0 - 1 .. i0 + 4 (i0 = 4q) of rows r - 1, r, r + 1 as three aligned
// dwords of the LDS-staged rows (each row staged with its edge columns replicated to columns -1 and
// dw, which turns jdsample.c's edge cases (i == 0, i == dw - 1) into the general formula), forms
// the column sums 3 * row r + neighbour row as packed 16-bit pairs, and the output pairs
// (3 * colsum(i) + colsum(i -+ 1) + 8 / 7) >> 4 of h2v2_fancy_upsample the same way.  Luma comes
// straight from the plane (8-byte loads).  Bit-exact with the general path: same integer formulas.
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
constexpr int kH2v2Pad = 8; // staged chroma row: [8 bytes: col -1 at 7][pw bytes][8 bytes: col dw]

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

// One staged chroma row's bytes i0 - 1 .. i0 + 4 as 16-bit pairs: P0 (i0-1, i0), P1 (i0+1, i0+2),
// P2 (i0+3, i0+4), Q0 (i0, i0+1), Q1 (i0+2, i0+3); `row` is 4-byte aligned at column i0 - 4.
struct ChromaCols {
    u16x2 p0, p1, p2, q0, q1;
};
__device__ __forceinline__ ChromaCols chroma_cols(const uint8_t* row)
{
    const uint32_t* w  = (const uint32_t*)row;
    const uint32_t  d0 = w[0], d1 = w[1], d2 = w[2];
    ChromaCols      c;
    c.p0 = as_u16x2(__builtin_amdgcn_perm(d1, d0, 0x0c040c03u));
    c.p1 = as_u16x2(__builtin_amdgcn_perm(d1, d1, 0x0c020c01u));
    c.p2 = as_u16x2(__builtin_amdgcn_perm(d2, d1, 0x0c040c03u));
    c.q0 = as_u16x2(__builtin_amdgcn_perm(d1, d1, 0x0c010c00u));
    c.q1 = as_u16x2(__builtin_amdgcn_perm(d1, d1, 0x0c030c02u));
    return c;
}

// h2v2_fancy_upsample of 8 output columns of one output row: e01 = (x0, x0 + 2), o01 = (x0 + 1,
// x0 + 3), e23 = (x0 + 4, x0 + 6), o23 = (x0 + 5, x0 + 7); `t3` = 3 * row r, `nb` the neighbour row.
struct ChromaOut {
    u16x2 e01, o01, e23, o23;
};
__device__ __forceinline__ ChromaOut chroma_row(const ChromaCols& t3, const ChromaCols& nb)
{
    const u16x2 three = {3, 3}, r8 = {8, 8}, r7 = {7, 7}, four = {4, 4};
    const u16x2 sp0 = t3.p0 + nb.p0, sp1 = t3.p1 + nb.p1, sp2 = t3.p2 + nb.p2;
    const u16x2 sq0 = t3.q0 + nb.q0, sq1 = t3.q1 + nb.q1;
    ChromaOut o;
    o.e01 = (sq0 * three + sp0 + r8) >> four;
    o.o01 = (sq0 * three + sp1 + r7) >> four;
    o.e23 = (sq1 * three + sp1 + r8) >> four;
    o.o23 = (sq1 * three + sp2 + r7) >> four;
    return o;
}

// jdcolor.c ycc_rgb_convert of one pixel, packed B | G << 8 | R << 16
__device__ __forceinline__ uint32_t ycc_bgr(int Y, int cb, int cr)
{
    cb -= 128, cr -= 128;
    const int r  = Y + ((91881 * cr + 32768) >> 16);
    const int g  = Y + ((-22554 * cb + 32768 + -46802 * cr) >> 16);
    const int bl = Y + ((116130 * cb + 32768) >> 16);
    return (uint32_t)min(max(bl, 0), 255) | (uint32_t)min(max(g, 0), 255) << 8 | (uint32_t)min(max(r, 0), 255) << 16;
}

// 8 BGR pixels of one output row to `o`: three 8-byte stores (aligned), six dwords, or bytes
__device__ __forceinline__ void store_bgr8(gp<uint8_t> o, const uint32_t (&p)[8], int n)
{
    uint32_t d[6];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        d[3 * h + 0] = p[4 * h] | p[4 * h + 1] << 24;
        d[3 * h + 1] = p[4 * h + 1] >> 8 | p[4 * h + 2] << 16;
        d[3 * h + 2] = p[4 * h + 2] >> 16 | p[4 * h + 3] << 8;
    }
    const uintptr_t a = (uintptr_t)o;
    if (n == 8 && (a & 7) == 0) {
        const gp<uint2> d2 = (gp<uint2>)o;
        d2[0] = make_uint2(d[0], d[1]), d2[1] = make_uint2(d[2], d[3]), d2[2] = make_uint2(d[4], d[5]);
    } else if (n == 8 && (a & 3) == 0) {
        const gp<uint32_t> d4 = (gp<uint32_t>)o;
#pragma unroll
        for (int e = 0; e < 6; e++) d4[e] = d[e];
    } else {
        for (int e = 0; e < 3 * n; e++) o[e] = (uint8_t)(d[e >> 2] >> (8 * (e & 3)));
    }
}

__device__ __forceinline__ void color_h2v2(const JpegImage& I, const JpegRows& R, uint8_t* lds)
{
    const int y0 = R.y0, y1 = R.y0 + R.rows - 1;
    // stage chroma rows [lo, hi] of both components, then replicate their edge columns
    int lo[2], n[2], lp[2], off[2];
    int o = 0;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const int k = c + 1;
        lo[c] = max((y0 >> 1) - 1, 0);
        n[c]  = min((y1 >> 1) + 1, I.dh[k] - 1) - lo[c] + 1;
        lp[c] = I.bw[k] * 8 + 2 * kH2v2Pad, off[c] = o;
        const gp<const uint2> src = (gp<const uint2>)(gaddr<const uint8_t>(I.planes[k]) + (size_t)lo[c] * (I.bw[k] * 8));
        const int per = I.bw[k]; // 8-byte words per row
        for (int e = threadIdx.x; e < n[c] * per; e += blockDim.x) {
            const int rr = e / per, w = e - rr * per;
            *(uint2*)(lds + o + rr * lp[c] + kH2v2Pad + w * 8) = src[e];
        }
        o += n[c] * lp[c];
    }
    __syncthreads();
    if (threadIdx.x < n[0] + n[1]) {
        const bool c1 = threadIdx.x >= n[0]; // (selects, not an index: the arrays stay in registers)
        const int  rr = threadIdx.x - (c1 ? n[0] : 0);
        uint8_t*   row = lds + (c1 ? off[1] + rr * lp[1] : rr * lp[0]) + kH2v2Pad;
        const int  dw  = c1 ? I.dw[2] : I.dw[1];
        row[-1] = row[0], row[dw] = row[dw - 1];
    }
    __syncthreads();

    const int W = I.W, H = I.H, groups = (W + 7) >> 3, pairs = (R.rows + 1) >> 1;
    const int pw0 = I.bw[0] * 8, dh1 = I.dh[1], dh2 = I.dh[2];
    const gp<const uint8_t> Yp  = gaddr<const uint8_t>(I.planes[0]);
    const gp<uint8_t>       out = gaddr<uint8_t>(I.out);
    const float rcp   = 1.0f / (float)groups;
    const int   total = groups * pairs;
    // the luma of the lane's next item is loaded before this one is computed
    auto luma = [&](int it, uint2& a, uint2& b) {
        const int pr = (int)(((float)it + 0.5f) * rcp), q = it - pr * groups;
        const int y = y0 + 2 * pr, x0 = q * 8;
        a = *(gp<const uint2>)(Yp + (size_t)y * pw0 + x0);
        b = *(gp<const uint2>)(Yp + (size_t)min(y + 1, H - 1) * pw0 + x0);
    };
    uint2 na = make_uint2(0, 0), nb = make_uint2(0, 0);
    if (threadIdx.x < total) luma(threadIdx.x, na, nb);
    for (int it = threadIdx.x; it < total; it += blockDim.x) {
        const uint2 ya = na, yv = nb;
        if (it + (int)blockDim.x < total) luma(it + blockDim.x, na, nb);
        const int pr = (int)(((float)it + 0.5f) * rcp), q = it - pr * groups;
        const int y = y0 + 2 * pr, x0 = q * 8, i0 = q * 4, r = y >> 1;
        ChromaOut ce[2], co[2]; // [chroma]: output row y (even), y + 1 (odd)
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int      dh   = c ? dh2 : dh1;
            const uint8_t* base = lds + off[c] + kH2v2Pad - 4 + i0;
            const ChromaCols m  = chroma_cols(base + (max(r - 1, 0) - lo[c]) * lp[c]);
            const ChromaCols t  = chroma_cols(base + (r - lo[c]) * lp[c]);
            const ChromaCols p  = chroma_cols(base + (min(r + 1, dh - 1) - lo[c]) * lp[c]);
            const u16x2      three = {3, 3};
            const ChromaCols t3 = {t.p0 * three, t.p1 * three, t.p2 * three, t.q0 * three, t.q1 * three};
            ce[c] = chroma_row(t3, m);
            co[c] = chroma_row(t3, p);
        }
        const int nx = min(8, W - x0);
#pragma unroll
        for (int v = 0; v < 2; v++) {
            if (v == 1 && y + 1 > y1) continue; // (the band's last row, or the image's)
            const uint2 yy = v ? yv : ya;
            const ChromaOut& cb = v ? co[0] : ce[0];
            const ChromaOut& cr = v ? co[1] : ce[1];
            const u16x2 bq[4] = {cb.e01, cb.o01, cb.e23, cb.o23}, rq[4] = {cr.e01, cr.o01, cr.e23, cr.o23};
            uint32_t px[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                // pixel e: even e -> e01/e23, odd -> o01/o23; pair half = (e >> 1) & 1
                const int      s  = (e >> 2) * 2 + (e & 1), h = (e >> 1) & 1;
                const uint32_t yw = e < 4 ? yy.x : yy.y;
                px[e] = ycc_bgr((int)((yw >> (8 * (e & 3))) & 0xff), (int)bq[s][h], (int)rq[s][h]);
            }
            store_bgr8(out + (size_t)(y + v) * I.out_stride + (size_t)x0 * 3, px, nx);
        }
    }
}

// A workgroup per band of output rows: the plane rows the band's upsampling reads are copied into
// LDS with coalesced 8-byte loads (jpeg_stage_rows bounds them), then color_rows.
__global__ __launch_bounds__(256) void jpeg_color(const JpegImage* __restrict__ imgs, const JpegRows* __restrict__ rows)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_b[];
    const JpegRows   R  = rows[blockIdx.x];
    const JpegImage& I  = imgs[R.img];
    if (I.ncomp == 3 && I.out_cn == 3 && I.up[0] == UP_FULL && I.up[1] == UP_H2V2 && I.up[2] == UP_H2V2 &&
        (R.y0 & 1) == 0) {
        color_h2v2(I, R, lds_b);
        return;
    }
    const int        nc = I.out_cn == 1 ? 1 : I.ncomp;
    const int        y1 = R.y0 + R.rows - 1;
    CompView         cv[3];
    int              off = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        CompView& c = cv[k];
        int       hi;
        comp_rows(I, k, R.y0, y1, c, hi);
        c.P = lds_b + off;
        if (k >= nc) continue;
        // stage plane rows [lo, hi]: whole rows of pw bytes (a multiple of 8) are contiguous
        const gp<const uint2> src = (gp<const uint2>)(gaddr<const uint8_t>(I.planes[k]) + (size_t)c.lo * c.pw);
        uint2*       dst = (uint2*)(lds_b + off);
        const int    n8  = (hi - c.lo + 1) * c.pw / 8;
        for (int e = threadIdx.x; e < n8; e += blockDim.x) dst[e] = src[e];
        off += (hi - c.lo + 1) * c.pw;
    }
    __syncthreads();
    color_rows(I, cv, R.y0, R.rows);
}

hipError_t launch_jpeg(const JpegImage* imgs, const JpegChunk* chunks, int n_chunks, const JpegRows* rows, int n_rows,
                       int color_lds, hipStream_t stream)
{
    if (n_chunks > 0) hipLaunchKernelGGL(jpeg_idct, dim3(n_chunks), dim3(kJpegIdctLanes), 0, stream, imgs, chunks);
    if (n_rows > 0) {
        if (color_lds > 64 * 1024) {
            const hipError_t e = hipFuncSetAttribute((const void*)jpeg_color, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     color_lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(jpeg_color, dim3(n_rows), dim3(256), (size_t)color_lds, stream, imgs, rows);
    }
    return hipGetLastError();
}

} // namespace aeon_hip
