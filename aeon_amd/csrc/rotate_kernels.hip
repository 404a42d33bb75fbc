// rotate_kernels.hip -- image::rotate (src/image.cpp:53-75) on the GPU: OpenCV 2.4 warpAffine
// about (cols/2, rows/2), INTER_LINEAR (images) or INTER_NEAREST (pixel masks), BORDER_CONSTANT 0,
// output the input's size.  A pre-pass: the rotated record lands in the slot scratch and the
// rest of transform_single_image reads it from there.
//
// Arithmetic (imgwarp.cpp WarpAffineInvoker + remapBilinear / remapNearest), per output pixel
// with the host-inverted matrix M (double, no FMA contraction -- built with -ffp-contract=off):
//   X = cvRound((M1*y + M2)*1024) + round_delta + cvRound(M0*x*1024)     (Y likewise: M4, M5, M3)
//   nearest: (X >> 10, Y >> 10); linear: (X >> 5 >> 5, Y >> 5 >> 5), fractions (X & 31, Y & 31),
//   weights (32-fy)(32-fx)*32 ... ({32767,0,0,1} at (0,0)), (sum + 2^14) >> 15, taps outside -> 0.
#include <hip/hip_runtime.h>

#include <cmath>

#include "aug_job.hpp"

namespace aeon_hip {

typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int cv_round_d(double v) { return (int)__builtin_rint(v); }
__device__ __forceinline__ int sat_short(int v) { return min(max(v, -32768), 32767); }

// One workgroup = a 64 x 32 tile of the output window.  The source pixels its taps can reach -- the
// bounding box of the tile's four corners mapped through M, plus the bilinear second tap -- are
// staged in LDS first as one word per pixel (bytes 0..cn-1, zero outside the image: BORDER_CONSTANT),
// so the per-pixel gathers are LDS reads and the global traffic is coalesced rows.  Lane l owns the
// 4 consecutive output pixels 4*(l%16) .. +3 of rows l/16 and l/16 + 16 and stores them as one
// 4*cn-byte group.  The LDS the launch asks for follows its steepest angle (rot_box_words): more
// workgroups per CU for small angles.  The per-row (X0, Y0) and per-column (adelta, bdelta) terms are warpAffine's own.
constexpr int kRotTX = 64, kRotTY = 32; // output tile (columns x rows)
constexpr int kRotMaxWords = 76 * 76;   // >= the source box of a tile at any angle (see rot_box_words)

struct RotMap {
    double M[6];
    int    rdelta, linear;
    __device__ __forceinline__ int X0(int y) const { return cv_round_d((M[1] * y + M[2]) * 1024) + rdelta; }
    __device__ __forceinline__ int Y0(int y) const { return cv_round_d((M[4] * y + M[5]) * 1024) + rdelta; }
    __device__ __forceinline__ int AD(int x) const { return cv_round_d(M[0] * x * 1024); }
    __device__ __forceinline__ int BD(int x) const { return cv_round_d(M[3] * x * 1024); }
    // first source tap of output pixel (x, y) from its fixed-point (X, Y) sums
    __device__ __forceinline__ int tap(int s) const { return linear ? sat_short(s >> 5 >> 5) : sat_short(s >> 10); }
};

// words: the launch's LDS capacity for the box (rot_box_words of its steepest angle).  CN: bytes per
// pixel of every job of the launch (1, 2 or 3: unrolled channel loops), 0 = each job's own.
template <int CN>
__global__ __launch_bounds__(256) void rotate_tiles(const RotJob* __restrict__ jobs, int words, int32_t* error)
{
    extern __shared__ uint32_t st[];
    __shared__ int box[4];
    const RotJob& R   = jobs[blockIdx.y];
    const int     tpr = (R.ow + kRotTX - 1) / kRotTX;
    if ((int)blockIdx.x >= tpr * ((R.oh + kRotTY - 1) / kRotTY)) return;
    const int tx0 = R.ox + (blockIdx.x % tpr) * kRotTX, ty0 = R.oy + (blockIdx.x / tpr) * kRotTY;
    const int tx1 = min(tx0 + kRotTX, R.ox + R.ow) - 1, ty1 = min(ty0 + kRotTY, R.oy + R.oh) - 1;
    const int W = R.w, H = R.h, cn = CN ? CN : R.cn, tid = threadIdx.x;
    RotMap    m;
    for (int k = 0; k < 6; k++) m.M[k] = R.M[k];
    m.linear = R.interp == 0;
    m.rdelta = m.linear ? 1024 / 32 / 2 : 1024 / 2;
    // source box: the taps are monotone in x and in y (each term rounded separately), so the
    // corners bound them; +1 for the bilinear second tap
    if (tid < 4) {
        const int x = (tid & 1) ? tx1 : tx0, y = (tid & 2) ? ty1 : ty0;
        box[tid] = (m.tap(m.X0(y) + m.AD(x)) & 0xffff) | (m.tap(m.Y0(y) + m.BD(x)) << 16);
    }
    __syncthreads();
    int bx0 = 1 << 30, by0 = 1 << 30, bx1 = -(1 << 30), by1 = -(1 << 30);
    for (int k = 0; k < 4; k++) {
        const int sx = (short)(box[k] & 0xffff), sy = box[k] >> 16;
        bx0 = min(bx0, sx), bx1 = max(bx1, sx), by0 = min(by0, sy), by1 = max(by1, sy);
    }
    bx1 += m.linear, by1 += m.linear;
    const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1, pitch = (bw + 3) & ~3; // pitch: whole 16-byte groups
    if (pitch * bh > words) { // cannot happen (the host sizes `words` for the launch's angles): flag it
        if (tid == 0) atomicOr(error, 64);
        return;
    }
    // stage: the box's 4-pixel groups, lane-strided.  Every load of a lane is issued before any is
    // used (buffer loads at kOOB return 0: the predication costs no branch): one 12-byte load per
    // group inside the image (BGR), byte loads for groups straddling its left / right edge (and for
    // 1- / 2-byte pixels); zero outside
    const auto src = __builtin_amdgcn_make_buffer_rsrc((void*)R.src_ptr, (short)0, R.stride * H, 0x00020000);
    const int  gpr = pitch >> 2, ng = gpr * bh;
    const float inv = 1.f / (float)gpr;
    constexpr uint32_t kOOB = 0x80000000u;
    constexpr int      kNG  = (kRotMaxWords / 4 + 255) / 256; // groups per lane (pitch * bh <= kRotMaxWords)
    u32x3 v[kNG];
    int   meta[kNG]; // box row | group << 12 | straddle flag << 30, -1 = none
#pragma unroll
    for (int i = 0; i < kNG; i++) {
        const int q = tid + i * 256;
        meta[i]     = -1;
        v[i]        = (u32x3){0, 0, 0};
        if (q >= ng) continue;
        const int  j = (int)(((float)q + 0.5f) * inv), g = q - j * gpr; // exact for q < 2^20
        const int  gy = by0 + j, gx = bx0 + 4 * g;
        const bool row_in = gy >= 0 && gy < H;
        const int  off = gy * R.stride + gx * cn;
        const bool fast = row_in && cn == 3 && gx >= 0 && gx + 3 < W && off + 12 <= R.stride * H;
        const bool none = !row_in || gx + 3 < 0 || gx >= W;
        meta[i]         = j | (g << 12) | ((!fast && !none) ? 1 << 30 : 0);
#ifdef AEON_HIP_EXP_ROT_NOSTAGE // development ablation: no source loads (wrong values)
        v[i] = (u32x3){(uint32_t)off, 0, 0};
        meta[i] &= (1 << 30) - 1;
#else
        v[i] = __builtin_amdgcn_raw_buffer_load_b96(src, fast ? (uint32_t)off : kOOB, 0, 0);
#endif
    }
#pragma unroll
    for (int i = 0; i < kNG; i++) {
        if (meta[i] < 0) continue;
        const int j = meta[i] & 0xfff, g4 = 4 * ((meta[i] >> 12) & 0xfff);
        uint32_t  w4[4];
        if (meta[i] >> 30) { // straddling an image edge: per byte, masked
            const int gy = by0 + j, gx = bx0 + g4;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int  x  = gx + k;
                const bool in = x >= 0 && x < W;
                w4[k]         = 0;
#pragma unroll
                for (int c = 0; c < (CN ? CN : 4); c++) {
                    if (c >= cn) break;
                    w4[k] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(src, in ? (uint32_t)(gy * R.stride + x * cn + c) : kOOB,
                                                                          0, 0) << (8 * c);
                }
            }
        } else { // 12 bytes BGR BGR BGR BGR -> four (B, G, R, 0) words (or zeros)
            w4[0] = v[i].x & 0xffffffu;
            w4[1] = __builtin_amdgcn_perm(v[i].y, v[i].x, 0x0C050403u);
            w4[2] = __builtin_amdgcn_perm(v[i].z, v[i].y, 0x0C040302u);
            w4[3] = v[i].z >> 8;
        }
        *(u32x4*)&st[j * pitch + g4] = (u32x4){w4[0], w4[1], w4[2], w4[3]}; // one ds_write_b128 per group
    }
    __syncthreads();
#ifdef AEON_HIP_EXP_ROT_NOCOMPUTE // development ablation: staging only
    return;
#endif
    // compute + store
    const int  ob  = R.ow * R.oh * cn;
    const auto dst = __builtin_amdgcn_make_buffer_rsrc((void*)R.out_ptr, (short)0, ob, 0x00020000);
    const int  x0  = tx0 + 4 * (tid & 15);
    if (x0 > tx1) return;
    int ad[4], bd[4];
#pragma unroll
    for (int k = 0; k < 4; k++) ad[k] = m.AD(x0 + k), bd[k] = m.BD(x0 + k);
    for (int y = ty0 + (tid >> 4); y <= ty1; y += 16) {
        const int X0 = m.X0(y), Y0 = m.Y0(y);
        uint32_t  px[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (!m.linear) {
                const int sx = m.tap(X0 + ad[k]) - bx0, sy = m.tap(Y0 + bd[k]) - by0;
                px[k]        = st[__mul24(sy, pitch) + sx];
                continue;
            }
            const int X = (X0 + ad[k]) >> 5, Y = (Y0 + bd[k]) >> 5;
            const int sx = sat_short(X >> 5) - bx0, sy = sat_short(Y >> 5) - by0;
            const int fx = X & 31, fy = Y & 31;
            // remapBilinear's 15-bit weights, (32767, 0, 0, 1) at (0, 0); they sum to 32768, so the
            // result never exceeds 255.  Per channel: the (tap, tap+1) byte pair of each row as two
            // u16 lanes (v_perm_b32) against the row's weight pair (v_dot2_u32_u16).
            // (24-bit multiplies: full rate; every factor here is < 2^12)
            const uint32_t gx = 32 - fx, gy = 32 - fy;
            uint32_t       w01 = (__umul24(__umul24(gy, gx), 32u)) | (__umul24(__umul24(gy, fx), 32u) << 16);
            uint32_t       w23 = (__umul24(__umul24(fy, gx), 32u)) | (__umul24(__umul24(fy, fx), 32u) << 16);
            if ((fx | fy) == 0) w01 = 32767u, w23 = 1u << 16;
            const int      a0  = __mul24(sy, pitch) + sx;
            const uint32_t p00 = st[a0], p01 = st[a0 + 1], p10 = st[a0 + pitch], p11 = st[a0 + pitch + 1];
            uint32_t       o   = 0;
#pragma unroll
            for (int c = 0; c < (CN ? CN : 4); c++) {
                if (c >= cn) break;
                const uint32_t sel = (uint32_t)c | (0x0Cu << 8) | ((4u + c) << 16) | (0x0Cu << 24);
                uint32_t       h   = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p01, p00, sel)),
                                                            __builtin_bit_cast(u16x2, w01), 1u << 14, false);
                h = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p11, p10, sel)),
                                           __builtin_bit_cast(u16x2, w23), h, false);
                o |= (h >> 15) << (8 * c);
            }
            px[k] = o;
        }
        const int nk  = min(4, tx1 + 1 - x0);
        const int off = ((y - R.oy) * R.ow + (x0 - R.ox)) * cn;
        if (nk == 4 && (off & 3) == 0 && cn == 3) {
            const u32x3 q = {px[0] | (px[1] << 24), (px[1] >> 8) | (px[2] << 16), (px[2] >> 16) | (px[3] << 8)};
            __builtin_amdgcn_raw_buffer_store_b96(q, dst, off, 0, 0);
        } else if (nk == 4 && (off & 3) == 0 && cn == 1) {
            __builtin_amdgcn_raw_buffer_store_b32(px[0] | (px[1] << 8) | (px[2] << 16) | (px[3] << 24), dst, off, 0, 0);
        } else {
            for (int k = 0; k < nk; k++)
#pragma unroll
                for (int c = 0; c < (CN ? CN : 4); c++)
                    if (c < cn) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(px[k] >> (8 * c)), dst, off + k * cn + c, 0, 0);
        }
    }
}

// image::expand: every canvas pixel is the record's pixel (x - ox, y - oy) or 0 outside it.
__global__ __launch_bounds__(256) void expand_records(const ExpandJob* __restrict__ jobs)
{
    const ExpandJob E  = jobs[blockIdx.y];
    const int       px = blockIdx.x * 256 + threadIdx.x;
    if (px >= E.ew * E.eh) return;
    const int      y = px / E.ew, x = px - y * E.ew;
    const int      sx = x - E.ox, sy = y - E.oy;
    const bool     in = sx >= 0 && sx < E.w && sy >= 0 && sy < E.h;
    const uint8_t* S  = (const uint8_t*)E.src_ptr + (size_t)sy * E.stride + (size_t)sx * E.cn;
    uint8_t*       D  = (uint8_t*)E.out_ptr + (size_t)px * E.cn;
    for (int c = 0; c < E.cn; c++) D[c] = in ? S[c] : 0;
}

hipError_t launch_expand(const ExpandJob* jobs, int n_jobs, int max_pixels, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    const dim3 grid((unsigned)((max_pixels + 255) / 256), (unsigned)n_jobs), block(256);
    hipLaunchKernelGGL(expand_records, grid, block, 0, stream, jobs);
    return hipGetLastError();
}

// Source-box words of one tile at `angle` degrees: its extents (TX|cos| + TY|sin|, TX|sin| + TY|cos|)
// + 1 for rounding at each end + 1 for the bilinear second tap.
int rot_box_words(int angle)
{
    const double a = angle * (3.14159265358979323846 / 180), c = std::fabs(std::cos(a)), s = std::fabs(std::sin(a));
    const int    w = (int)std::ceil(kRotTX * c + kRotTY * s) + 4, h = (int)std::ceil(kRotTX * s + kRotTY * c) + 4;
    return ((w + 3) & ~3) * h; // rows of whole 4-pixel groups
}

// max_tiles: the most output tiles of any job's window; words: max rot_box_words of its angles;
// cn: the jobs' common bytes per pixel, 0 if they differ
hipError_t launch_rotate(const RotJob* jobs, int n_jobs, int max_tiles, int words, int cn, int32_t* error, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    if (words > kRotMaxWords) return hipErrorInvalidValue;
    const dim3   grid((unsigned)max_tiles, (unsigned)n_jobs), block(256);
    const size_t lds = (size_t)words * 4;
    switch (cn) {
    case 3: hipLaunchKernelGGL(rotate_tiles<3>, grid, block, lds, stream, jobs, words, error); break;
    case 1: hipLaunchKernelGGL(rotate_tiles<1>, grid, block, lds, stream, jobs, words, error); break;
    case 2: hipLaunchKernelGGL(rotate_tiles<2>, grid, block, lds, stream, jobs, words, error); break;
    default: hipLaunchKernelGGL(rotate_tiles<0>, grid, block, lds, stream, jobs, words, error); break;
    }
    return hipGetLastError();
}

} // namespace aeon_hip
