// jpeg_kernels.hip -- GPU half of the JPEG decode stage (see jpeg.hpp), bit-exact with libjpeg's
// defaults as cv::imdecode runs them under aeon's image::extractor::extract (etl_image.cpp:83-99).
//
// jpeg_idct: eight lanes per 8x8 block.  They scatter the block's non-zero coefficients (zigzag
// mask + values), dequantised, into its LDS slot (a mask byte each), then run jidctint.c's
// jpeg_idct_islow (LL&M, CONST_BITS 13, PASS1_BITS 2; the post-IDCT range limit of jdmaster.c,
// x & 1023 wrap) -- integer multiply-adds only -- a column each, then a row each, and each lane
// writes its output row of the block into the component plane (one 8-byte store).
// jpeg_color: one lane per 4 output pixels of each of kJpegRowsPerWg rows: each component sampled
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

__device__ __forceinline__ uint32_t idct_limit(int x)
{
    const int i = x & 1023;
    return i < 128 ? (uint32_t)(i + 128) : (i < 512 ? 255u : (i < 896 ? 0u : (uint32_t)(i - 896)));
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
// every block's descriptor, then every column gather -- lane j takes column j straight from the
// sparse stream (coefficient at natural n = r*8 + j present iff its zigzag bit is set; its value
// index = the set bits below it): no zero fill, no scatter, all loads in flight together -- then
// per block pass 1 in registers, a transpose through the wave's own LDS region (no workgroup
// barrier) and pass 2 on row j.  Slot stride 66 dwords: lane (g, j) of pass 1 writes bank
// (2g + 8r + j) % 64 -- conflict-free per wave.
constexpr int kSlot = 66;

__global__ __launch_bounds__(kJpegIdctLanes) void jpeg_idct(const JpegImage* __restrict__ imgs,
                                                            const JpegChunk* __restrict__ chunks)
{
    constexpr int G = kJpegIdctLanes / 8; // lane groups per workgroup
    __shared__ int slot[G * kSlot];
    const JpegChunk  C  = chunks[blockIdx.x];
    const JpegImage& I  = imgs[C.img];
    const int        k  = C.comp;
    const int        g = threadIdx.x >> 3, j = threadIdx.x & 7;
    const gp<const JpegBlock> blocks = gaddr<const JpegBlock>(I.blocks[k]) + C.first;
    const gp<const int16_t>   vals   = gaddr<const int16_t>(I.values);
    const gp<const int16_t>   dense  = gaddr<const int16_t>(I.dvals[k]);
    JpegBlock        B[kJpegIdctUnroll];
#pragma unroll
    for (int u = 0; u < kJpegIdctUnroll; u++) B[u] = blocks[min(g + u * G, C.count - 1)];
    int qv[8];
#pragma unroll
    for (int r = 0; r < 8; r++) qv[r] = I.q[k][r * 8 + j];
    // pass 1 inputs: column j of every block, dequantised (jidctint.c DEQUANTIZE = coef * quantval);
    // a GPU-decoded file's coefficients sit at their zigzag slot of the block's 64
    int col[kJpegIdctUnroll][8];
    if (dense) {
#pragma unroll
        for (int u = 0; u < kJpegIdctUnroll; u++) {
            const gp<const int16_t> bv = dense + (size_t)(C.first + min(g + u * G, C.count - 1)) * 64;
#pragma unroll
            for (int r = 0; r < 8; r++) { // unconditional loads, the mask zeroes the stale slots
                const int z = kZzInv[r * 8 + j];
                col[u][r]   = ((int)bv[z] * qv[r]) & -(int)((B[u].mask >> z) & 1);
            }
        }
    } else {
#pragma unroll
        for (int u = 0; u < kJpegIdctUnroll; u++)
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int z = kZzInv[r * 8 + j];
                col[u][r]   = 0;
                if ((B[u].mask >> z) & 1)
                    col[u][r] = (int)vals[B[u].val_off + __builtin_popcountll(B[u].mask & ((1ull << z) - 1))] * qv[r];
            }
    }
    int* s = slot + g * kSlot;
    const int bw = I.bw[k];
#pragma unroll
    for (int u = 0; u < kJpegIdctUnroll; u++) {
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
            const int bx = b % bw, by = b / bw;
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

// A workgroup per band of output rows: the plane rows the band's upsampling reads are copied into
// LDS with coalesced 8-byte loads (jpeg_stage_rows bounds them), then color_rows.
__global__ __launch_bounds__(256) void jpeg_color(const JpegImage* __restrict__ imgs, const JpegRows* __restrict__ rows)
{
    extern __shared__ uint8_t lds_b[];
    const JpegRows   R  = rows[blockIdx.x];
    const JpegImage& I  = imgs[R.img];
    const int        nc = I.out_cn == 1 ? 1 : I.ncomp;
    const int        y1 = R.y0 + R.rows - 1;
    CompView         cv[3];
    int              off = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (k >= nc) break;
        CompView& c = cv[k];
        int       hi;
        comp_rows(I, k, R.y0, y1, c, hi);
        c.P = lds_b + off;
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
