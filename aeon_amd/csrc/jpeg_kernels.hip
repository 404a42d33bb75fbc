// jpeg_kernels.hip -- GPU half of the JPEG decode stage (see jpeg.hpp), bit-exact with libjpeg's
// defaults as cv::imdecode runs them under aeon's image::extractor::extract (etl_image.cpp:83-99).
//
// jpeg_idct: one lane per 8x8 block.  The lane scatters its block's non-zero coefficients
// (zigzag mask + values), dequantised, into a private LDS slot, pulls the 64 values into VGPRs and
// runs jidctint.c's jpeg_idct_islow (LL&M, CONST_BITS 13, PASS1_BITS 2; the post-IDCT range limit of
// jdmaster.c, x & 1023 wrap) -- integer multiply-adds only -- then writes the 8 output rows of the
// block into its component plane (two dword stores per row).
// jpeg_color: one lane per output pixel column of kJpegRowsPerWg rows: each component sampled
// through jdsample.c's upsampler (h2v1 / h1v2 / h2v2 fancy triangle filters, context rows
// replicated at the edges as jdmainct.c does; box replication for the other ratios and for
// components narrower than 3 samples), then jdcolor.c ycc_rgb_convert (16-bit fixed point) and the
// BGR store of the decoded record into the augmentation stage's source arena.
#include <hip/hip_runtime.h>

#include "jpeg.hpp"

namespace aeon_hip {

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

// Slot stride 65 dwords: lane l's word w sits in bank (65 l + w) % 64 -- conflict-free per word.
constexpr int kSlot = 65;

__global__ __launch_bounds__(kJpegIdctLanes) void jpeg_idct(const JpegImage* __restrict__ imgs,
                                                            const JpegChunk* __restrict__ chunks)
{
    __shared__ int slot[kJpegIdctLanes * kSlot];
    __shared__ int qt[64];
    const JpegChunk C  = chunks[blockIdx.x];
    const JpegImage& I = imgs[C.img];
    const int        k = C.comp;
    if (threadIdx.x < 64) qt[threadIdx.x] = I.q[k][threadIdx.x];
    int* s = slot + threadIdx.x * kSlot;
#pragma unroll
    for (int w = 0; w < 64; w++) s[w] = 0;
    __syncthreads();
    if ((int)threadIdx.x >= C.count) return;
    const int        b  = C.first + threadIdx.x;
    const int        bw = I.bw[k];
    const JpegBlock  B  = ((const JpegBlock*)I.blocks[k])[b];
    const int16_t*   v  = (const int16_t*)I.values + B.val_off;
    uint64_t         m  = B.mask;
    // jdhuff.c leaves coefficients in natural order; DEQUANTIZE = coef * quantval (jidctint.c)
    for (int j = 0; m; j++) {
        const int z = __builtin_ctzll(m);
        m &= m - 1;
        const int nat = kZz[z];
        s[nat]        = (int)v[j] * qt[nat];
    }
    int c[64];
#pragma unroll
    for (int w = 0; w < 64; w++) c[w] = s[w];
    // pass 1: columns (in c[r*8 + col]) -> ws, descaled by CONST_BITS - PASS1_BITS
    int ws[64];
#pragma unroll
    for (int col = 0; col < 8; col++) {
        int in[8], out[8];
#pragma unroll
        for (int r = 0; r < 8; r++) in[r] = c[r * 8 + col];
        llm8<11, false>(in, out);
#pragma unroll
        for (int r = 0; r < 8; r++) ws[r * 8 + col] = out[r];
    }
    // pass 2: rows, descaled by CONST_BITS + PASS1_BITS + 3, range limited
    uint8_t* plane = (uint8_t*)I.planes[k];
    const int pitch = bw * 8;
    const int bx = b % bw, by = b / bw;
    uint8_t*  o  = plane + (size_t)(by * 8) * pitch + bx * 8;
#pragma unroll
    for (int r = 0; r < 8; r++) {
        int out[8];
        llm8<18, true>(&ws[r * 8], out);
        const uint32_t lo = idct_limit(out[0]) | idct_limit(out[1]) << 8 | idct_limit(out[2]) << 16 | idct_limit(out[3]) << 24;
        const uint32_t hi = idct_limit(out[4]) | idct_limit(out[5]) << 8 | idct_limit(out[6]) << 16 | idct_limit(out[7]) << 24;
        *(uint2*)(o + (size_t)r * pitch) = make_uint2(lo, hi);
    }
}

// Sample (x, y) of the image from component k's plane through libjpeg's upsampler.
__device__ __forceinline__ int upsampled(const JpegImage& I, int k, int x, int y)
{
    const uint8_t* P  = (const uint8_t*)I.planes[k];
    const int      pw = I.bw[k] * 8;
    const int      hf = I.hmax / I.hs[k], vf = I.vmax / I.vs[k];
    auto at = [&](int cx, int cy) { return (int)P[(size_t)cy * pw + cx]; };
    if (hf == 1 && vf == 1) return at(x, y);
    const int  dw = I.dw[k], dh = I.dh[k];
    const bool fancy = dw > 2;
    if (hf == 2 && vf == 1 && fancy) { // h2v1_fancy_upsample
        const int i = x >> 1;
        if ((x & 1) == 0) return i == 0 ? at(0, y) : (at(i, y) * 3 + at(i - 1, y) + 1) >> 2;
        return i == dw - 1 ? at(i, y) : (at(i, y) * 3 + at(i + 1, y) + 2) >> 2;
    }
    if (hf == 1 && vf == 2 && fancy) { // h1v2_fancy_upsample (libjpeg-turbo)
        const int r = y >> 1, v = y & 1;
        const int nb = v == 0 ? max(r - 1, 0) : min(r + 1, dh - 1);
        return (at(x, r) * 3 + at(x, nb) + (v ? 2 : 1)) >> 2;
    }
    if (hf == 2 && vf == 2 && fancy) { // h2v2_fancy_upsample
        const int r = y >> 1, v = y & 1;
        const int nb = v == 0 ? max(r - 1, 0) : min(r + 1, dh - 1);
        const int i  = x >> 1;
        auto cs = [&](int ci) { return at(ci, r) * 3 + at(ci, nb); };
        const int t = cs(i);
        if ((x & 1) == 0) return i == 0 ? (t * 4 + 8) >> 4 : (t * 3 + cs(i - 1) + 8) >> 4;
        return i == dw - 1 ? (t * 4 + 7) >> 4 : (t * 3 + cs(i + 1) + 7) >> 4;
    }
    return at(x / hf, y / vf); // h2v1_upsample / h2v2_upsample / int_upsample
}

__global__ __launch_bounds__(256) void jpeg_color(const JpegImage* __restrict__ imgs, const JpegRows* __restrict__ rows)
{
    const JpegRows   R = rows[blockIdx.x];
    const JpegImage& I = imgs[R.img];
    uint8_t*         out = (uint8_t*)I.out;
    for (int y = R.y0; y < R.y0 + R.rows; y++)
        for (int x = threadIdx.x; x < I.W; x += blockDim.x) {
            uint8_t* o = out + (size_t)y * I.out_stride + (size_t)x * I.out_cn;
            const int Y = upsampled(I, 0, x, y);
            if (I.out_cn == 1) {
                o[0] = (uint8_t)Y;
            } else if (I.ncomp == 1) {
                o[0] = o[1] = o[2] = (uint8_t)Y;
            } else {
                const int cb = upsampled(I, 1, x, y) - 128, cr = upsampled(I, 2, x, y) - 128;
                const int r  = Y + ((91881 * cr + 32768) >> 16);
                const int g  = Y + ((-22554 * cb + 32768 + -46802 * cr) >> 16);
                const int b  = Y + ((116130 * cb + 32768) >> 16);
                o[0] = (uint8_t)min(max(b, 0), 255);
                o[1] = (uint8_t)min(max(g, 0), 255);
                o[2] = (uint8_t)min(max(r, 0), 255);
            }
        }
}

hipError_t launch_jpeg(const JpegImage* imgs, const JpegChunk* chunks, int n_chunks, const JpegRows* rows, int n_rows,
                       hipStream_t stream)
{
    if (n_chunks > 0) hipLaunchKernelGGL(jpeg_idct, dim3(n_chunks), dim3(kJpegIdctLanes), 0, stream, imgs, chunks);
    if (n_rows > 0) hipLaunchKernelGGL(jpeg_color, dim3(n_rows), dim3(256), 0, stream, imgs, rows);
    return hipGetLastError();
}

} // namespace aeon_hip
