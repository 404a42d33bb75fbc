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

#include "aug_job.hpp"

namespace aeon_hip {

__device__ __forceinline__ int cv_round_d(double v) { return (int)__builtin_rint(v); }
__device__ __forceinline__ int sat_short(int v) { return min(max(v, -32768), 32767); }

__global__ __launch_bounds__(256) void rotate_records(const RotJob* __restrict__ jobs)
{
    const RotJob R  = jobs[blockIdx.y];
    const int    W  = R.w, H = R.h, cn = R.cn;
    const int    px = blockIdx.x * 256 + threadIdx.x;
    if (px >= W * H) return;
    const int      y = px / W, x = px - y * W;
    const uint8_t* S = (const uint8_t*)R.src_ptr;
    uint8_t*       D = (uint8_t*)R.out_ptr + (size_t)px * cn;
    auto tap = [&](int xx, int yy, int c) -> int {
        return (xx >= 0 && xx < W && yy >= 0 && yy < H) ? S[(size_t)yy * R.stride + xx * cn + c] : 0;
    };
    const int rdelta = R.interp == 0 ? 1024 / 32 / 2 : 1024 / 2;
    const int X0 = cv_round_d((R.M[1] * y + R.M[2]) * 1024) + rdelta;
    const int Y0 = cv_round_d((R.M[4] * y + R.M[5]) * 1024) + rdelta;
    const int ad = cv_round_d(R.M[0] * x * 1024), bd = cv_round_d(R.M[3] * x * 1024);
    if (R.interp != 0) {
        const int sx = sat_short((X0 + ad) >> 10), sy = sat_short((Y0 + bd) >> 10);
        for (int c = 0; c < cn; c++) D[c] = (uint8_t)tap(sx, sy, c);
        return;
    }
    const int X = (X0 + ad) >> 5, Y = (Y0 + bd) >> 5;
    const int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
    const int fx = X & 31, fy = Y & 31;
    int       w0, w1, w2, w3;
    if (fx == 0 && fy == 0) {
        w0 = 32767, w1 = 0, w2 = 0, w3 = 1;
    } else {
        w0 = (32 - fy) * (32 - fx) * 32, w1 = (32 - fy) * fx * 32;
        w2 = fy * (32 - fx) * 32, w3 = fy * fx * 32;
    }
    for (int c = 0; c < cn; c++) {
        const int v = tap(sx, sy, c) * w0 + tap(sx + 1, sy, c) * w1 + tap(sx, sy + 1, c) * w2 +
                      tap(sx + 1, sy + 1, c) * w3;
        D[c] = (uint8_t)min(max((v + (1 << 14)) >> 15, 0), 255);
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

hipError_t launch_rotate(const RotJob* jobs, int n_jobs, int max_pixels, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    const dim3 grid((unsigned)((max_pixels + 255) / 256), (unsigned)n_jobs), block(256);
    hipLaunchKernelGGL(rotate_records, grid, block, 0, stream, jobs);
    return hipGetLastError();
}

} // namespace aeon_hip
