// resize_kernels.hip -- cv::resize with INTER_CUBIC, INTER_LANCZOS4 and INTER_AREA (OpenCV 2.4.9
// imgwarp.cpp), the interpolation methods aeon's image::config accepts besides LINEAR / NEAREST
// (src/image.cpp:30-36; image::resize :93-106, image::resize_short :118-127).  A pre-pass per
// record: the resized window lands in the slot scratch as HWC uint8 and the record's tile job copies
// it through the photometric stages and the loader (stage.cpp plan_image).
//
// Arithmetic (oracle/aeon_oracle.cpp resize_cv restates the same; parity unpinned -- aeon's tests
// hold no output of these methods):
//  * CUBIC / LANCZOS4 / INTER_AREA's bilinear emulation: resizeGeneric_ -- per destination column
//    the clamped sx and ksize 11-bit coefficients, per row the raw sy with rows clipped; the
//    horizontal pass is exact int; the vertical pass is VResizeCubicVec_32s8u's float sums for the
//    elements the SSE2 build covers 8 at a time, VResizeLinearVec_32s8u's for the bilinear emulation,
//    FixedPtCast<int, uchar, 22> over wrapping int32 sums for the rest (all of Lanczos4).
//  * INTER_AREA, both axes downscaled: integer factors -> resizeAreaFast_ (2x2 -> (a+b+c+d+2)>>2,
//    else saturate_cast<uchar>(sum * (1.f / area))); otherwise resizeArea_ over computeResizeAreaTab:
//    float sums in table order, horizontal then vertical.
// A workgroup takes one tile (rows [y0, y0 + TR) x columns [x0, x0 + CW) of a record's window): the
// column and row taps go to LDS, then the horizontal pass of every source row the tile's rows touch
// (each staged source row read from global memory once per tile, int or float sums in LDS), then
// the vertical pass writes the tile.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "aug_job.hpp"

namespace aeon_hip {

namespace {

__device__ __forceinline__ int sat_u8(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int sat_s16(int v) { return min(max(v, -32768), 32767); }
__device__ __forceinline__ int coef_q(float c) { return sat_s16((int)__builtin_rintf(c * 2048)); }

__device__ __forceinline__ void interpolate_cubic(float x, float* c)
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

__device__ __forceinline__ int ksize_of(int m) { return m == GR_CUBIC ? 4 : (m == GR_LANCZOS4 ? 8 : 2); }

// First element of a W-element row on the scalar tail of the vertical pass (SSE2 build).
__device__ __forceinline__ int simd_end(int ksize, int W)
{
    int x = 0;
    if (ksize == 2) {
        x = W >= 16 ? (W / 16) * 16 : 0;
        while (x < W - 4) x += 4;
    } else if (ksize == 4) {
        x = W >= 8 ? (W / 8) * 8 : 0;
    }
    return x;
}

// resize-source pixel (u, v) (the crop, add_padding's zero border applied), channel c
__device__ __forceinline__ int src_px(const ResizeJob& J, int u, int v, int c)
{
    if (J.padded) {
        u += J.shift_x, v += J.shift_y;
        if (u < 0 || v < 0 || u >= J.crop_w || v >= J.crop_h) return 0;
    }
    return ((const uint8_t*)J.src_ptr)[(size_t)(J.crop_y + v) * J.src_stride + (size_t)(J.crop_x + u) * J.cn + c];
}

// K-tap filters: destination column dx -> (clamped sx, K coefficients), cv::resize's set-up
__device__ __forceinline__ void col_taps(const ResizeJob& J, int dx, int* t)
{
    const int K = ksize_of(J.method);
    float     fx;
    int       sx;
    if (J.method == GR_LINEAR_AREA) {
        sx = (int)floor(dx * J.scale_x);
        fx = (float)((dx + 1) - (sx + 1) * J.inv_x);
        fx = fx <= 0 ? 0.f : fx - (float)(int)floorf(fx);
    } else {
        fx = (float)((dx + 0.5) * J.scale_x - 0.5);
        sx = (int)floorf(fx);
        fx -= (float)sx;
    }
    if (sx < 0) fx = 0.f, sx = 0;
    if (sx >= J.crop_w - 1) fx = 0.f, sx = J.crop_w - 1;
    float c[4];
    if (K == 4) interpolate_cubic(fx, c);
    else c[0] = 1.f - fx, c[1] = fx;
    t[0] = sx;
    for (int k = 0; k < K; k++) t[1 + k] = coef_q(c[k]);
}
__device__ __forceinline__ void row_taps(const ResizeJob& J, int dy, int* t)
{
    const int K = ksize_of(J.method);
    float     fy;
    int       sy;
    if (J.method == GR_LINEAR_AREA) {
        sy = (int)floor(dy * J.scale_y);
        fy = (float)((dy + 1) - (sy + 1) * J.inv_y);
        fy = fy <= 0 ? 0.f : fy - (float)(int)floorf(fy);
    } else {
        fy = (float)((dy + 0.5) * J.scale_y - 0.5);
        sy = (int)floorf(fy);
        fy -= (float)sy;
    }
    float c[4];
    if (K == 4) interpolate_cubic(fy, c);
    else c[0] = 1.f - fy, c[1] = fy;
    t[0] = sy;
    for (int k = 0; k < K; k++) t[1 + k] = coef_q(c[k]);
}

// computeResizeAreaTab's entries of destination index d: consecutive source indices from t[0], t[1]
// of them, weights (float bits) from t[2]
__device__ __forceinline__ void area_taps(int ssize, double scale, int d, int* t, int amax, int32_t* error)
{
    const double fs1 = d * scale, fs2 = fs1 + scale;
    const double cell = min(scale, ssize - fs1);
    int          s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
    s2 = min(s2, ssize - 1);
    s1 = min(s1, s2);
    int n = 0;
    t[0]  = s1;
    if (s1 - fs1 > 1e-3) t[0] = s1 - 1, t[2 + n++] = __float_as_int((float)((s1 - fs1) / cell));
    for (int s = s1; s < s2 && n < amax; s++) t[2 + n++] = __float_as_int((float)(1.0 / cell));
    if (fs2 - s2 > 1e-3 && n < amax) t[2 + n++] = __float_as_int((float)(min(min(fs2 - s2, 1.), cell) / cell));
    if (s2 - s1 + 2 > amax) atomicOr(error, 128); // any lane whose taps were cut (the host sizes amax: never)
    t[1] = n;
}

} // namespace

// grid (tiles, jobs); LDS: xt[CW][xs] | yt[TR][xs] | H[NR][CW][cn] words
__global__ __launch_bounds__(256) void resize_generic(const ResizeJob* __restrict__ jobs, const uint8_t* __restrict__ table,
                                                      int TR, int CW, int NR, int xs, int amax, int32_t* error)
{
    extern __shared__ int lds_w[];
    const ResizeJob J = jobs[blockIdx.y];
    if ((int)blockIdx.x >= J.tiles) return;
    const int tid = threadIdx.x, nt = blockDim.x, cn = J.cn;
    const int ty = blockIdx.x / J.tiles_x, tx = blockIdx.x - ty * J.tiles_x;
    const int x0 = tx * CW, y0 = ty * TR;
    const int nx = min(CW, J.win_w - x0), ny = min(TR, J.win_h - y0);
    uint8_t*  out = (uint8_t*)J.out_ptr;

    if (J.method == GR_AREA_FAST) { // resizeAreaFast_: integer box, no staging
        const bool  fast2 = J.isx == 2 && J.isy == 2 && (cn == 1 || cn == 3 || cn == 4);
        const float scale = 1.f / (J.isx * J.isy);
        for (int q = tid; q < ny * nx * cn; q += nt) {
            const int r = q / (nx * cn), e = q - r * nx * cn, i = e / cn, c = e - i * cn;
            const int dx = J.win_x + x0 + i, dy = J.win_y + y0 + r;
            int       sum = 0;
            for (int y = 0; y < J.isy; y++)
                for (int x = 0; x < J.isx; x++) sum += src_px(J, dx * J.isx + x, dy * J.isy + y, c);
            out[((size_t)(y0 + r) * J.win_w + x0 + i) * cn + c] =
                (uint8_t)(fast2 ? (sum + 2) >> 2 : sat_u8((int)__builtin_rintf((float)sum * scale)));
        }
        return;
    }

    const bool area = J.method == GR_AREA;
    const int  K = ksize_of(J.method), k2 = K / 2;
    int*       xt = lds_w;
    int*       yt = xt + CW * xs;
    int*       H  = yt + TR * xs;
    // taps of the tile's columns and rows
    for (int i = tid; i < nx; i += nt) {
        int* t = xt + i * xs;
        if (area) area_taps(J.crop_w, J.scale_x, J.win_x + x0 + i, t, amax, error);
        else if (J.method == GR_LANCZOS4) {
            const GrTap g = ((const GrTap*)(table + J.coef_x))[x0 + i];
            t[0]          = g.s;
            for (int k = 0; k < 8; k++) t[1 + k] = g.c[k];
        } else col_taps(J, J.win_x + x0 + i, t);
    }
    for (int r = tid; r < ny; r += nt) {
        int* t = yt + r * xs;
        if (area) area_taps(J.crop_h, J.scale_y, J.win_y + y0 + r, t, amax, error);
        else if (J.method == GR_LANCZOS4) {
            const GrTap g = ((const GrTap*)(table + J.coef_y))[y0 + r];
            t[0]          = g.s;
            for (int k = 0; k < 8; k++) t[1 + k] = g.c[k];
        } else row_taps(J, J.win_y + y0 + r, t);
    }
    __syncthreads();
    // the source rows the tile touches (row taps are monotone)
    const int* tf = yt;
    const int* tl = yt + (ny - 1) * xs;
    const int  r_lo = area ? tf[0] : min(max(tf[0] - k2 + 1, 0), J.crop_h - 1);
    const int  r_hi = area ? tl[0] + tl[1] - 1 : min(max(tl[0] + k2, 0), J.crop_h - 1);
    const int  nr   = r_hi - r_lo + 1;
    if (nr > NR) {
        if (tid == 0) atomicOr(error, 128);
        return;
    }
    // horizontal pass: H[r][i][c] (int sums, or float bits for INTER_AREA)
    for (int q = tid; q < nr * nx; q += nt) {
        const int  r = q / nx, i = q - r * nx, v = r_lo + r;
        const int* t = xt + i * xs;
        for (int c = 0; c < cn; c++) {
            if (area) {
                float b = 0.f;
                for (int e = 0; e < t[1]; e++) b = b + (float)src_px(J, t[0] + e, v, c) * __int_as_float(t[2 + e]);
                H[(r * CW + i) * cn + c] = __float_as_int(b);
            } else {
                int acc = 0;
                for (int j = 0; j < K; j++) acc += src_px(J, min(max(t[0] - k2 + 1 + j, 0), J.crop_w - 1), v, c) * t[1 + j];
                H[(r * CW + i) * cn + c] = acc;
            }
        }
    }
    __syncthreads();
    // vertical pass
    const int W  = J.dst_w * cn;
    const int xv = simd_end(K, W);
    for (int q = tid; q < ny * nx * cn; q += nt) {
        const int  r = q / (nx * cn), e = q - r * nx * cn, i = e / cn, c = e - i * cn;
        const int* t = yt + r * xs;
        int        v;
        if (area) {
            float sum = 0.f;
            for (int k = 0; k < t[1]; k++)
                sum = sum + __int_as_float(t[2 + k]) * __int_as_float(H[((t[0] + k - r_lo) * CW + i) * cn + c]);
            v = sat_u8((int)__builtin_rintf(sum));
        } else {
            const int x = (J.win_x + x0 + i) * cn + c; // element of the full destination row
            auto      h = [&](int k) { return H[((min(max(t[0] - k2 + 1 + k, 0), J.crop_h - 1) - r_lo) * CW + i) * cn + c]; };
            if (x < xv && K == 2) { // VResizeLinearVec_32s8u
                const int m = sat_s16(((sat_s16(h(0) >> 4) * t[1]) >> 16) + ((sat_s16(h(1) >> 4) * t[2]) >> 16));
                v           = sat_u8(sat_s16(m + 2) >> 2);
            } else if (x < xv && K == 4) { // VResizeCubicVec_32s8u, SSE's order of operations
                const float sc = 1.f / (2048 * 2048);
                float       s  = (float)h(0) * ((float)t[1] * sc) + (float)h(1) * ((float)t[2] * sc);
                s              = s + (float)h(2) * ((float)t[3] * sc);
                s              = s + (float)h(3) * ((float)t[4] * sc);
                v              = sat_u8(sat_s16((int)__builtin_rintf(s)));
            } else { // FixedPtCast<int, uchar, 22>, int32 sums wrapping
                uint32_t acc = 0;
                for (int k = 0; k < K; k++) acc += (uint32_t)h(k) * (uint32_t)t[1 + k];
                v = sat_u8((int32_t)(acc + (1u << 21)) >> 22);
            }
        }
        out[((size_t)(y0 + r) * J.win_w + x0 + i) * cn + c] = (uint8_t)v;
    }
}

hipError_t launch_resize_generic(const ResizeJob* jobs, const uint8_t* table, int n_jobs, int max_tiles, int TR, int CW,
                                 int NR, int xs, int amax, int cn_max, int32_t* error, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    const size_t lds = ((size_t)CW * xs + (size_t)TR * xs + (size_t)NR * CW * cn_max) * 4;
    hipLaunchKernelGGL(resize_generic, dim3((unsigned)max_tiles, (unsigned)n_jobs), dim3(256), lds, stream, jobs, table, TR,
                       CW, NR, xs, amax, error);
    return hipGetLastError();
}

} // namespace aeon_hip
