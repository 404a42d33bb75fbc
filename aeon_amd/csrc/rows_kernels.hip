// rows_kernels.hip -- the plain single-pass record path (aeon's C2 / C5-image shape) as a streaming
// kernel with no LDS staging.
//
// crop -> cv::resize INTER_LINEAR (OpenCV 2.4 fixed point, SSE2 vertical formula) -> flip ->
// loader::load (BGR->RGB, HWC->CHW, standardize) for 3-channel uint8 records into float32 CHW
// planes (aeon src/etl_image.cpp:146-202, 246-341; src/image.cpp:93-106).  The tile kernel
// (augment_kernels.hip) stages a band's source rows in LDS behind workgroup barriers, one staging
// buffer per workgroup; here every lane reads its own taps straight from the source (8-byte
// loads at the exact, unaligned byte offset of each tap pair, served by L1/L2 after the first
// touch) and there is no barrier after the prologue, so the CU's many independent waves cover
// the load latency and the store stream never waits for a staging phase.
//
// Workgroup = one band of TR output rows of one record (4 waves; wave w takes rows w, w + 4, ...);
// lane = one group of 4 consecutive output columns (its taps stay in registers for the band); the
// grid is not persistent (the dispatcher refills CUs).  Two rows are loaded before either is
// computed.  Rows whose 8-byte windows would cross the end of the record's bytes take per-byte
// loads (a buffer access straddling the range returns zero as a whole).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "aug_job.hpp"

namespace aeon_hip {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

constexpr int kRowsThreads = 256;
constexpr int kJobDwords   = 32; // AugJob fields read here all lie in its first 128 bytes
static_assert(__builtin_offsetof(AugJob, flip) + 4 <= 4 * kJobDwords, "AugJob prefix");

__device__ __forceinline__ int sat_s16(int v) { return min(max(v, -32768), 32767); }
__device__ __forceinline__ int rnd(float v) { return (int)__builtin_rintf(v); }

// OpenCV 2.4 resizeGeneric_ INTER_LINEAR taps (as xcoef / ycoef in augment_kernels.hip)
struct Tap {
    int s, w0, w1;
};
__device__ __forceinline__ Tap xtap(int dx, double scale, int sw)
{
    float fx = (float)((dx + 0.5) * scale - 0.5);
    int   sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) fx = 0.f, sx = 0;
    if (sx + 1 >= sw) fx = 0.f, sx = sw - 1;
    return Tap{sx, sat_s16(rnd((1.f - fx) * 2048.f)), sat_s16(rnd(fx * 2048.f))};
}
struct YTap {
    int r0, r1, b0, b1;
};
__device__ __forceinline__ YTap ytap(int dy, double scale, int sh)
{
    float fy = (float)((dy + 0.5) * scale - 0.5);
    int   sy = (int)floorf(fy);
    fy -= (float)sy;
    return YTap{min(max(sy, 0), sh - 1), min(max(sy + 1, 0), sh - 1), sat_s16(rnd((1.f - fy) * 2048.f)),
                sat_s16(rnd(fy * 2048.f))};
}

// The 8 bytes at source byte offset b (unaligned): pixel S[sx] in bytes 0-2, S[sx+1] in 3-5.
__device__ __forceinline__ u32x2 load8(__amdgpu_buffer_rsrc_t r, int b)
{
#if defined(ROWS_EXP_ALIGNED) // development ablation: 8-byte aligned loads (wrong values)
    return __builtin_amdgcn_raw_buffer_load_b64(r, b & ~7, 0, 0);
#elif defined(ROWS_EXP_NOLOAD) // development ablation: no source loads (wrong values)
    return (u32x2){(uint32_t)b, (uint32_t)b * 3u};
#elif defined(ROWS_EXP_DWORDS) // three aligned dwords + alignbyte
    const int      a4 = b & ~3, sh = (b & 3) * 8;
    const uint32_t d0 = __builtin_amdgcn_raw_buffer_load_b32(r, a4, 0, 0), d1 = __builtin_amdgcn_raw_buffer_load_b32(r, a4 + 4, 0, 0),
                   d2 = __builtin_amdgcn_raw_buffer_load_b32(r, a4 + 8, 0, 0);
    return (u32x2){(uint32_t)(((uint64_t)d1 << 32 | d0) >> sh), (uint32_t)(((uint64_t)d2 << 32 | d1) >> sh)};
#elif defined(ROWS_EXP_X3) // one aligned dwordx3 + alignbyte
    const int   a4 = b & ~3, sh = (b & 3) * 8;
    const u32x3 d  = __builtin_amdgcn_raw_buffer_load_b96(r, a4, 0, 0);
    return (u32x2){(uint32_t)(((uint64_t)d.y << 32 | d.x) >> sh), (uint32_t)(((uint64_t)d.z << 32 | d.y) >> sh)};
#else
    return __builtin_amdgcn_raw_buffer_load_b64(r, b, 0, 0);
#endif
}
// The same, byte by byte (rows at the end of the record's range).
__device__ __forceinline__ u32x2 load8_bytes(__amdgpu_buffer_rsrc_t r, int b)
{
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) lo |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, b + i, 0, 0) << (8 * i);
#pragma unroll
    for (int i = 0; i < 2; i++) hi |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, b + 4 + i, 0, 0) << (8 * i);
    return (u32x2){lo, hi};
}

// HResizeLinear + VResizeLinearVec_32s8u of one channel of one output pixel, as the tile kernel's
// resize_px: (S[sx], S[sx+1]) of each row gathered into two u16 lanes by v_perm_b32, one
// v_dot2_u32_u16 with (a0, a1), then ((H0>>4)*b0 >> 16) + ((H1>>4)*b1 >> 16) + 2, i.e. 4x the
// pixel plus 0..3 (the LUT index without further shifts).
template <int C>
__device__ __forceinline__ uint32_t resize_ch(u32x2 p0, u32x2 p1, u16x2 w, int b0, int b1)
{
    constexpr uint32_t sel = (uint32_t)C | (0x0Cu << 8) | ((3u + C) << 16) | (0x0Cu << 24);
    const uint32_t     H0  = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p0.y, p0.x, sel)), w, 0u, false);
    const uint32_t     H1  = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p1.y, p1.x, sel)), w, 0u, false);
    const uint32_t     t0  = (uint32_t)__mul24((int)(H0 >> 4), b0) + (2u << 16);
    const uint32_t     t1  = (uint32_t)__mul24((int)(H1 >> 4), b1);
    return (t0 >> 16) + (t1 >> 16);
}

} // namespace

#ifndef ROWS_WAVES
#define ROWS_WAVES 1
#endif
__global__ __launch_bounds__(kRowsThreads) __attribute__((amdgpu_waves_per_eu(ROWS_WAVES))) void augment_rows(LaunchArgs a)
{
    __shared__ uint32_t sjob[kJobDwords];
    __shared__ float    slut[3 * 256];
    const int tid  = threadIdx.x;
    const int t    = blockIdx.x;
    const int job  = t / a.max_tiles;
    const int band = t - job * a.max_tiles;
    if (tid < kJobDwords) {
        const auto jr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.jobs + job), (short)0, 4 * kJobDwords, 0x00020000);
        // a pinned host table is read through to the host (sc0 sc1): the host rewrote the slot
        sjob[tid] = a.jobs_host ? __builtin_amdgcn_raw_buffer_load_b32(jr, 4 * tid, 0, 17)
                                : __builtin_amdgcn_raw_buffer_load_b32(jr, 4 * tid, 0, 0);
    }
    for (int i = tid; i < 3 * 256; i += kRowsThreads) slut[i] = a.lut[i];
    __syncthreads();
    const auto ju = [&](int off) { return (uint32_t)__builtin_amdgcn_readfirstlane(sjob[off / 4]); };
    const auto ji = [&](int off) { return (int)ju(off); };
    const auto jd = [&](int off) {
        return __builtin_bit_cast(double, (uint64_t)ju(off) | ((uint64_t)ju(off + 4) << 32));
    };
    const auto jp = [&](int off) { return (uint64_t)ju(off) | ((uint64_t)ju(off + 4) << 32); };
#define JO(f) (int)__builtin_offsetof(AugJob, f)
    const int TR    = a.rows_per_tile;
    const int win_w = ji(JO(win_w)), win_h = ji(JO(win_h));
    const int y0    = band * TR;
    const int nrows = min(TR, win_h - y0);
    if (nrows <= 0) return;
    const double scale_x = jd(JO(scale_x)), scale_y = jd(JO(scale_y));
    const int    crop_x = ji(JO(crop_x)), crop_y = ji(JO(crop_y)), crop_w = ji(JO(crop_w)), crop_h = ji(JO(crop_h));
    const int    win_x = ji(JO(win_x)), win_y = ji(JO(win_y));
    const int    stride = ji(JO(src_stride)), flip = ji(JO(flip));
    const int    src_bytes = ji(JO(src_bytes));
    const int    plane     = win_w * win_h;
    const auto   srs = __builtin_amdgcn_make_buffer_rsrc((void*)jp(JO(src_ptr)), (short)0, src_bytes, 0x00020000);
    const auto   ors = __builtin_amdgcn_make_buffer_rsrc((void*)jp(JO(out_ptr)), (short)0, 12 * plane, 0x00020000);
#undef JO
    const int lane = tid & 63, wave = tid >> 6;
    const int gpr  = win_w >> 2; // whole 4-pixel groups (the host routes other widths elsewhere)
    // a row's loads reach at most this many bytes past the row start (taps are monotone in dx)
    const int reach = (crop_x + xtap(win_x + win_w - 1, scale_x, crop_w).s) * 3 + 8;
    const int oc0 = a.bgr_to_rgb ? 2 : 0, oc2 = 2 - oc0; // output planes of source channels 0 / 2

    for (int cg = lane; cg < gpr; cg += 64) {
        const int ox0 = 4 * cg;
        int       off[4];
        u16x2     w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int x  = flip ? win_w - 1 - (ox0 + k) : ox0 + k;
            const Tap c  = xtap(win_x + x, scale_x, crop_w);
            off[k]       = (crop_x + c.s) * 3;
            w[k]         = (u16x2){(uint16_t)c.w0, (uint16_t)c.w1};
        }
        auto emit = [&](int y, const YTap& v, const u32x2 (&p0)[4], const u32x2 (&p1)[4]) {
            uint32_t s[4][3];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                s[k][0] = resize_ch<0>(p0[k], p1[k], w[k], v.b0, v.b1);
                s[k][1] = resize_ch<1>(p0[k], p1[k], w[k], v.b0, v.b1);
                s[k][2] = resize_ch<2>(p0[k], p1[k], w[k], v.b0, v.b1);
            }
            const int idx = y * win_w + ox0;
            const int ocs[3] = {oc0, 1, oc2};
#pragma unroll
            for (int c = 0; c < 3; c++) {
#ifdef ROWS_EXP_NOLUT // development ablation: no LUT reads (wrong values)
                const u32x4 q = {s[0][c], s[1][c], s[2][c], s[3][c]};
#else
                const u32x4 q = {__float_as_uint(slut[c * 256 + (s[0][c] >> 2)]), __float_as_uint(slut[c * 256 + (s[1][c] >> 2)]),
                                 __float_as_uint(slut[c * 256 + (s[2][c] >> 2)]), __float_as_uint(slut[c * 256 + (s[3][c] >> 2)])};
#endif
                __builtin_amdgcn_raw_buffer_store_b128(q, ors, (ocs[c] * plane + idx) * 4, 0, 2 /* nt */);
            }
        };
        auto load_row = [&](const YTap& v, u32x2 (&p0)[4], u32x2 (&p1)[4]) {
            const int r0 = (crop_y + v.r0) * stride, r1 = (crop_y + v.r1) * stride;
            if (r1 + reach <= src_bytes) { // r1 >= r0
#pragma unroll
                for (int k = 0; k < 4; k++) p0[k] = load8(srs, r0 + off[k]), p1[k] = load8(srs, r1 + off[k]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) p0[k] = load8_bytes(srs, r0 + off[k]), p1[k] = load8_bytes(srs, r1 + off[k]);
            }
        };
        int r = wave;
        for (; r + 4 < nrows; r += 8) { // two rows in flight
            const YTap va = ytap(win_y + y0 + r, scale_y, crop_h), vb = ytap(win_y + y0 + r + 4, scale_y, crop_h);
            u32x2      a0[4], a1[4], b0[4], b1[4];
            load_row(va, a0, a1);
            load_row(vb, b0, b1);
            emit(y0 + r, va, a0, a1);
            emit(y0 + r + 4, vb, b0, b1);
        }
        if (r < nrows) {
            const YTap va = ytap(win_y + y0 + r, scale_y, crop_h);
            u32x2      a0[4], a1[4];
            load_row(va, a0, a1);
            emit(y0 + r, va, a0, a1);
        }
    }
}

hipError_t launch_rows(const LaunchArgs& a, int grid, hipStream_t stream, hipEvent_t start, hipEvent_t stop)
{
    if (start || stop) {
        void* args[1] = {(void*)&a};
        return hipExtLaunchKernel((const void*)augment_rows, dim3(grid), dim3(kRowsThreads), args, 0, stream, start,
                                  stop, 0);
    }
    hipLaunchKernelGGL(augment_rows, dim3(grid), dim3(kRowsThreads), 0, stream, a);
    return hipGetLastError();
}

} // namespace aeon_hip
