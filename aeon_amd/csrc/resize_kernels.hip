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
// column and row taps go to LDS, the source rows and columns the tile touches are staged in LDS (read
// from global memory once per tile), then the horizontal pass (int or float sums in LDS), then the
// vertical pass writes the tile.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <type_traits>

#include "aug_job.hpp"

// (development: AEON_RG_SKIP bits drop the horizontal pass (1), the vertical pass / stores (2) or the
// staging (4) -- wrong outputs, phase timing only)
#ifndef AEON_RG_SKIP
#define AEON_RG_SKIP 0
#endif
#ifndef AEON_SEP_SCHED // resize_sep: a row's taps read together up to this K (K = 8's 32 loads in flight: 150+ VGPRs)
#define AEON_SEP_SCHED 4
#endif

namespace aeon_hip {

namespace {

__device__ __forceinline__ int sat_u8(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int sat_s16(int v) { return min(max(v, -32768), 32767); }
// 24-bit signed multiply-add, full rate (|operands| < 2^23; the sum wraps).  (Not inline asm: the
// compiler schedules no load across an asm statement, so each element's LDS reads waited for the previous
// element's multiply-adds.)
__device__ __forceinline__ int mad_i24(int a, int b, int c) { return (int)((uint32_t)__mul24(a, b) + (uint32_t)c); }
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
    return ((const __attribute__((address_space(1))) uint8_t*)J.src_ptr)[(size_t)(J.crop_y + v) * J.src_stride +
                                                                        (size_t)(J.crop_x + u) * J.cn + c];
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

// The loader for a final_out job (stage.cpp plan_image: no photometric stage, f32 output): element e
// of window row y (pixel e / cn, source channel e % cn) -> cv::flip, BGR->RGB, the standardize LUT (in
// LDS, [source channel][value]), stored into the output item's plane (channel-major) or pixel.
__device__ __forceinline__ void store_final(const ResizeJob& J, const float* lut, int bgr, int chm, int y, int x0, int e0,
                                            int nb, uint32_t word)
{
    const auto o  = (__attribute__((address_space(1))) float*)J.out_ptr;
    const int  cn = J.cn;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = e0 + q;
        if (e >= nb) break;
        const int px = e / cn, c = e - px * cn;
        const int x  = x0 + px;
        const int ox = J.flip ? J.win_w - 1 - x : x;
        const int oc = bgr ? 2 - c : c;
        const int i  = chm ? oc * J.out_plane + y * J.out_pitch + ox : (y * J.out_pitch + ox) * cn + oc;
        o[i]         = lut[c * 256 + ((word >> (8 * q)) & 0xff)];
    }
}

// store_final for 4 consecutive pixels x, x + 1, ... (n of them valid) of source channel c: one float4
// into the channel's plane when the 4 output elements are contiguous and 16-byte aligned (reversed
// when flipped), element stores otherwise.
__device__ __forceinline__ void store_planar(const ResizeJob& J, const float* lut, int bgr, int chm, int y, int x, int c, int n,
                                             uint32_t word)
{
    typedef float f32x4 __attribute__((ext_vector_type(4)));
    const auto o  = (__attribute__((address_space(1))) float*)J.out_ptr;
    const int  cn = J.cn, oc = bgr ? 2 - c : c;
    float      v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = lut[c * 256 + ((word >> (8 * q)) & 0xff)];
    if (chm && n >= 4) {
        const int  lo = J.flip ? J.win_w - 1 - (x + 3) : x; // the lowest of the 4 output columns
        const int  i  = oc * J.out_plane + y * J.out_pitch + lo;
        const auto p  = o + i;
        if (((uintptr_t)p & 15) == 0) {
            const f32x4 q4 = J.flip ? (f32x4){v[3], v[2], v[1], v[0]} : (f32x4){v[0], v[1], v[2], v[3]};
            __builtin_nontemporal_store(q4, (__attribute__((address_space(1))) f32x4*)p);
            return;
        }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q >= n) break;
        const int ox = J.flip ? J.win_w - 1 - (x + q) : x + q;
        o[chm ? oc * J.out_plane + y * J.out_pitch + ox : (y * J.out_pitch + ox) * cn + oc] = v[q];
    }
}

// grid (tiles, jobs); LDS: xt[CW][xs] | yt[TR][xs] | H[NR][CW * cn] words | S[NR][SW] bytes | LUT.
// S holds the tile's source rows [r_lo, r_hi] x columns [u_lo, u_hi] as src_px gives them (add_padding's
// zero border applied while staging), so both passes read LDS only: the horizontal pass one (row,
// column) per lane with the column's taps in registers, the vertical pass 4 consecutive output bytes
// per lane (one dword store) -- an element's H word is row * CW * cn + its byte index in the row.
__global__ __launch_bounds__(256) void resize_generic(const ResizeJob* __restrict__ jobs, const uint8_t* __restrict__ table,
                                                      int TR, int CW, int NR, int xs, int amax, int SW, const float* lutg,
                                                      int bgr, int chm, int32_t* error)
{
    extern __shared__ int lds_w[];
    const ResizeJob J = jobs[blockIdx.y];
    if ((int)blockIdx.x >= J.tiles) return;
    const int tid = threadIdx.x, nt = blockDim.x, cn = J.cn;
    const int ty = blockIdx.x / J.tiles_x, tx = blockIdx.x - ty * J.tiles_x;
    const int x0 = tx * CW, y0 = ty * TR;
    const int nx = min(CW, J.win_w - x0), ny = min(TR, J.win_h - y0);
    // global (not flat) pointers: a flat store counts on the LDS counter too, so the next LDS read's
    // wait would also wait for the store to reach memory
    const auto out = (__attribute__((address_space(1))) uint8_t*)J.out_ptr;

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
    const int  rowH = CW * cn; // H words per staged row
    int*       xt = lds_w;
    int*       yt = xt + CW * xs;
    int*       H  = yt + TR * xs;
    uint8_t*   S  = (uint8_t*)(H + NR * rowH);
    float*     lut = (float*)(S + NR * SW); // (final_out jobs)
    if (J.final_out)
        for (int i = tid; i < 768; i += nt) lut[i] = lutg[i];
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
    // the source rows and columns the tile touches (taps are monotone)
    const int* tf = yt;
    const int* tl = yt + (ny - 1) * xs;
    const int  r_lo = area ? tf[0] : min(max(tf[0] - k2 + 1, 0), J.crop_h - 1);
    const int  r_hi = area ? tl[0] + tl[1] - 1 : min(max(tl[0] + k2, 0), J.crop_h - 1);
    const int  nr   = r_hi - r_lo + 1;
    const int* cf   = xt;
    const int* cl   = xt + (nx - 1) * xs;
    const int  u_lo = area ? cf[0] : min(max(cf[0] - k2 + 1, 0), J.crop_w - 1);
    const int  u_hi = area ? cl[0] + cl[1] - 1 : min(max(cl[0] + k2, 0), J.crop_w - 1);
    const int  sb   = (u_hi - u_lo + 1) * cn; // staged bytes per row
    const bool staged = SW > 0; // (0: the host found no room for the staging -- large downscales)
    if (nr > NR || (staged && sb > SW)) {
        if (tid == 0) atomicOr(error, 128);
        return;
    }
    // staging: S[r][(u - u_lo) * cn + c] = src_px(u, r_lo + r, c), 4 bytes per lane and step; (row,
    // chunk) advanced incrementally (no divisions per step).  A staged byte b of row v is the source
    // byte (u_lo + shift_x) * cn + b of that row's crop, zero outside it when padded.
    if (staged && !(AEON_RG_SKIP & 4)) {
        const uint8_t* src  = (const uint8_t*)J.src_ptr + (size_t)J.crop_x * cn;
        const int      nch  = (sb + 3) >> 2, total = nr * nch;
        const int      dr   = nt / nch, dc = nt - dr * nch;
        const int      sx0  = (u_lo + (J.padded ? J.shift_x : 0)) * cn, rowb = J.crop_w * cn;
        int            r = tid / nch, ch = tid - r * nch;
        // kBatch steps' loads issued before their LDS writes (one memory latency per batch, not per step)
        constexpr int kBatch = 8;
        for (int q0 = tid; q0 < total; q0 += kBatch * nt) {
            uint32_t w[kBatch];
            int      at[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                w[u] = 0, at[u] = -1;
                {
                    // unconditional loads from clamped (valid) addresses, zeroed after: no branch
                    // around a load, so the batch's loads stay in flight together
                    const bool qv  = q0 + u * nt < total;
                    const int  rr  = min(r, nr - 1);
                    const int  v   = r_lo + rr + (J.padded ? J.shift_y : 0);
                    const bool vin = qv && (!J.padded || (v >= 0 && v < J.crop_h));
                    const auto row = (const __attribute__((address_space(1))) uint8_t*)(
                        src + (size_t)(J.crop_y + min(max(v, 0), J.crop_h - 1)) * J.src_stride);
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const int      b  = ch * 4 + k;
                        const int      bo = sx0 + b;
                        const bool     ok = b < sb && vin && (!J.padded || (bo >= 0 && bo < rowb));
                        const uint32_t x  = row[min(max(bo, 0), rowb - 1)];
                        w[u] |= (ok ? x : 0u) << (8 * k);
                    }
                    at[u] = qv ? rr * SW + ch * 4 : -1;
                }
                r += dr, ch += dc;
                if (ch >= nch) ch -= nch, r++;
            }
#pragma unroll
            for (int u = 0; u < kBatch; u++)
                if (at[u] >= 0) *(uint32_t*)(S + at[u]) = w[u];
        }
    }
    __syncthreads();
    // horizontal pass: H[r][i * cn + c] (int sums, or float bits for INTER_AREA); lane -> column i,
    // rows r, r + nt / nx, ... (its column's taps loaded once)
    {
        const int per = max(nt / nx, 1);
        const int i = tid % nx, r0 = tid / nx;
        if (r0 < per && tid < per * nx && !(AEON_RG_SKIP & 1)) {
            const int* t = xt + i * xs;
            if (area) {
                const int n = t[1], u0 = t[0] - u_lo;
                for (int r = r0; r < nr; r += per) {
                    const uint8_t* row = S + r * SW;
                    for (int c = 0; c < cn; c++) {
                        float b = 0.f;
                        for (int e = 0; e < n; e++)
                            b = b + (float)(staged ? row[(u0 + e) * cn + c] : src_px(J, t[0] + e, r_lo + r, c)) *
                                        __int_as_float(t[2 + e]);
                        H[r * rowH + i * cn + c] = __float_as_int(b);
                    }
                }
            } else if (!staged) {
                for (int r = r0; r < nr; r += per)
                    for (int c = 0; c < cn; c++) {
                        int acc = 0;
                        for (int j = 0; j < K; j++)
                            acc += src_px(J, min(max(t[0] - k2 + 1 + j, 0), J.crop_w - 1), r_lo + r, c) * t[1 + j];
                        H[r * rowH + i * cn + c] = acc;
                    }
            } else {
                int off[8], cf8[8];
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    off[j] = j < K ? (min(max(t[0] - k2 + 1 + j, 0), J.crop_w - 1) - u_lo) * cn : 0;
                    cf8[j] = j < K ? t[1 + j] : 0;
                }
                for (int r = r0; r < nr; r += per) {
                    const uint8_t* row = S + r * SW;
                    for (int c = 0; c < cn; c++) {
                        int acc = 0;
                        if (K == 4) {
#pragma unroll
                            for (int j = 0; j < 4; j++) acc += (int)row[off[j] + c] * cf8[j];
                        } else {
                            for (int j = 0; j < K; j++) acc += (int)row[off[j] + c] * cf8[j];
                        }
                        H[r * rowH + i * cn + c] = acc;
                    }
                }
            }
        }
    }
    __syncthreads();
    // vertical pass: 4 consecutive bytes of an output row per lane
    const int W   = J.dst_w * cn;
    const int xv  = simd_end(K, W);
    const int nb  = nx * cn;          // output bytes of a tile row
    const int nq  = (nb + 3) >> 2;    // dword groups per tile row
    const int xb0 = (J.win_x + x0) * cn; // the tile's first element in the full destination row
    for (int q = tid; q < ny * nq && !(AEON_RG_SKIP & 2); q += nt) {
        const int  r = q / nq, e0 = (q - r * nq) * 4;
        const int* t = yt + r * xs;
        uint32_t   word = 0;
        int        vals[4];
#pragma unroll
        for (int k4 = 0; k4 < 4; k4++) {
            const int e = min(e0 + k4, nb - 1);
            int       v;
            if (area) {
                float sum = 0.f;
                for (int k = 0; k < t[1]; k++) sum = sum + __int_as_float(t[2 + k]) * __int_as_float(H[(t[0] + k - r_lo) * rowH + e]);
                v = sat_u8((int)__builtin_rintf(sum));
            } else {
                const int x = xb0 + e; // element of the full destination row
                auto      h = [&](int k) { return H[(min(max(t[0] - k2 + 1 + k, 0), J.crop_h - 1) - r_lo) * rowH + e]; };
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
            vals[k4] = v;
            word |= (uint32_t)v << (8 * k4);
        }
        if (J.final_out) {
            store_final(J, lut, bgr, chm, y0 + r, x0, e0, nb, word);
            continue;
        }
        const auto dst = out + ((size_t)(y0 + r) * J.win_w + x0) * cn + e0;
        if (e0 + 4 <= nb && ((uintptr_t)dst & 3) == 0) {
            *(__attribute__((address_space(1))) uint32_t*)dst = word;
        } else {
            for (int k4 = 0; k4 < 4 && e0 + k4 < nb; k4++) dst[k4] = (uint8_t)vals[k4];
        }
    }
}

// The separable fixed-K methods (CUBIC K = 4, LANCZOS4 K = 8, INTER_AREA's bilinear emulation K = 2),
// one workgroup per band of TR output rows x CW columns: the band's source rows staged in LDS as above,
// then each lane owns 4 consecutive output bytes of the band's rows and walks the rows in order,
// keeping the K horizontal sums of its 4 elements it last used in registers (a new source row's sums
// are computed only when the row window moves onto it; the window position is uniform over the
// workgroup, so those branches are too).  No horizontal-sum array in LDS: the workgroup needs only the
// staged bytes and the taps, so several bands share a CU and their latencies overlap.  Same
// arithmetic as resize_generic, element for element.
// Each staged row sits kSepPadL bytes into its SW-byte slot: room for the replicated left border (at
// most K/2 - 1 pixels), as the slot's end has room for the right one (at most K/2), so every tap of an
// element is its first tap's staged byte + j * cn -- no per-tap clamp (cv::resize's border replicate).
constexpr int kSepPadL = 16;

// f(integral_constant<int, d>) for a workgroup-uniform d in 1..K (0: nothing)
template <int K, typename F>
__device__ __forceinline__ void sep_shift(int d, F&& f)
{
    if (d == 1) return f(std::integral_constant<int, 1>{});
    if (d == 2) return f(std::integral_constant<int, 2>{});
    if constexpr (K > 2) {
        if (d == 3) return f(std::integral_constant<int, 3>{});
        if (d == 4) return f(std::integral_constant<int, 4>{});
    }
    if constexpr (K > 4) {
        if (d == 5) return f(std::integral_constant<int, 5>{});
        if (d == 6) return f(std::integral_constant<int, 6>{});
        if (d == 7) return f(std::integral_constant<int, 7>{});
        if (d == 8) return f(std::integral_constant<int, 8>{});
    }
}

// CN: the jobs' channel count when it is 3 (the taps' LDS offsets immediates), else 0 (J.cn).
// AREA: resizeArea_ (both axes downscaled, non-integer): K = the most taps of a destination index
// (computeResizeAreaTab's entries, area_taps), float weights zero-padded to K -- exact, as every
// product is >= +0 and adding +0 changes no sum -- horizontal sums from 0 in tap order, the vertical sum
// beta0 * h0 + beta1 * h1 + ..., cvRound: ResizeArea_Invoker's arithmetic, element for element.
template <int K, int CN, bool AREA = false>
__global__ __launch_bounds__(256) void resize_sep(const ResizeJob* __restrict__ jobs, const uint8_t* __restrict__ table, int TR,
                                                  int CW, int NR, int SW, const float* lutg, int bgr, int chm, int32_t* error)
{
    extern __shared__ int lds_w[];
    const ResizeJob J = jobs[blockIdx.y];
    if ((int)blockIdx.x >= J.tiles) return;
    constexpr int k2 = AREA ? 1 : K / 2, xs = (AREA ? 2 : 1) + K; // (area: t[0] first index, t[1] taps, weights)
    const int     tid = threadIdx.x, nt = blockDim.x, cn = CN ? CN : J.cn;
    const int     ty = blockIdx.x / J.tiles_x, tx = blockIdx.x - ty * J.tiles_x;
    const int     x0 = tx * CW, y0 = ty * TR;
    const int     nx = min(CW, J.win_w - x0), ny = min(TR, J.win_h - y0);
    const auto    out = (__attribute__((address_space(1))) uint8_t*)J.out_ptr;
    int*          xt  = lds_w;
    int*          yt  = xt + CW * xs;
    uint8_t*      S   = (uint8_t*)lds_w + ((CW + TR) * xs * 4 + 15) / 16 * 16; // (16-aligned rows)
    float*        lut = (float*)(S + NR * SW);                                 // (final_out jobs)
    if (J.final_out)
        for (int i = tid; i < 768; i += nt) lut[i] = lutg[i];
    for (int i = tid; i < nx; i += nt) {
        int* t = xt + i * xs;
        if (AREA) {
            area_taps(J.crop_w, J.scale_x, J.win_x + x0 + i, t, K, error);
        } else if (K == 8) {
            const GrTap g = ((const GrTap*)(table + J.coef_x))[x0 + i];
            t[0]          = g.s;
            for (int k = 0; k < 8; k++) t[1 + k] = g.c[k];
        } else {
            col_taps(J, J.win_x + x0 + i, t);
        }
    }
    for (int r = tid; r < ny; r += nt) {
        int* t = yt + r * xs;
        if (AREA) {
            area_taps(J.crop_h, J.scale_y, J.win_y + y0 + r, t, K, error);
        } else if (K == 8) {
            const GrTap g = ((const GrTap*)(table + J.coef_y))[y0 + r];
            t[0]          = g.s;
            for (int k = 0; k < 8; k++) t[1 + k] = g.c[k];
        } else {
            row_taps(J, J.win_y + y0 + r, t);
        }
    }
    __syncthreads();
    const int r_lo = AREA ? yt[0] : min(max(yt[0] - k2 + 1, 0), J.crop_h - 1);
    const int r_hi = AREA ? yt[(ny - 1) * xs] + yt[(ny - 1) * xs + 1] - 1 : min(max(yt[(ny - 1) * xs] + k2, 0), J.crop_h - 1);
    const int nr   = r_hi - r_lo + 1;
    const int u_lo = AREA ? xt[0] : min(max(xt[0] - k2 + 1, 0), J.crop_w - 1);
    const int u_hi = AREA ? xt[(nx - 1) * xs] + xt[(nx - 1) * xs + 1] - 1 : min(max(xt[(nx - 1) * xs] + k2, 0), J.crop_w - 1);
    const int sb   = (u_hi - u_lo + 1) * cn;
    if (nr > NR || (J.padded ? sb : ((sb + 30) >> 4) * 16) + kSepPadL + 16 > SW || (CN && J.cn != CN)) {
        if (tid == 0) atomicOr(error, 128);
        return;
    }
    // Non-padded jobs: each staged row is the 16-byte-aligned blocks covering its bytes (one
    // dwordx4 load per block; a 16-byte-aligned block holding one byte of the row never leaves that
    // byte's page, so the over-read is always mapped), the row's first byte at S[r * SW + its
    // address & 15].  Padded jobs: byte by byte, the zero border applied (as resize_generic's).
    const uint64_t rowa0 = J.src_ptr + (uint64_t)J.crop_y * J.src_stride + (uint64_t)(J.crop_x + u_lo) * cn;
    if (AEON_RG_SKIP & 4) {
    } else if (!J.padded) {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const int     nblk = (sb + 15 + 15) >> 4; // blocks of the worst-aligned row
        const int     total = nr * nblk;
        constexpr int kBatch = 4;
        for (int q0 = tid; q0 < total; q0 += kBatch * nt) {
            u32x4 w[kBatch];
            int   at[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                const int      q  = min(q0 + u * nt, total - 1);
                const int      r  = q / nblk, b = q - r * nblk;
                const uint64_t a  = rowa0 + (uint64_t)(r_lo + r) * J.src_stride;
                const uint64_t a0 = a & ~(uint64_t)15;
                const int      bl = (int)((((a + sb - 1) & ~(uint64_t)15) - a0) >> 4); // the row's last block
                w[u]  = *(const __attribute__((address_space(1))) u32x4*)(a0 + (uint64_t)min(b, bl) * 16);
                at[u] = q0 + u * nt < total && b <= bl ? r * SW + kSepPadL + b * 16 : -1;
            }
#pragma unroll
            for (int u = 0; u < kBatch; u++)
                if (at[u] >= 0) *(u32x4*)(S + at[u]) = w[u];
        }
    } else { // staging (as resize_generic's)
        const uint8_t* src = (const uint8_t*)J.src_ptr + (size_t)J.crop_x * cn;
        const int      nch = (sb + 3) >> 2, total = nr * nch;
        const int      dr = nt / nch, dc = nt - dr * nch;
        const int      sx0 = (u_lo + (J.padded ? J.shift_x : 0)) * cn, rowb = J.crop_w * cn;
        int            r = tid / nch, ch = tid - r * nch;
        constexpr int  kBatch = 8;
        for (int q0 = tid; q0 < total; q0 += kBatch * nt) {
            uint32_t w[kBatch];
            int      at[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                const bool qv  = q0 + u * nt < total;
                const int  rr  = min(r, nr - 1);
                const int  v   = r_lo + rr + (J.padded ? J.shift_y : 0);
                const bool vin = qv && (!J.padded || (v >= 0 && v < J.crop_h));
                const auto row = (const __attribute__((address_space(1))) uint8_t*)(
                    src + (size_t)(J.crop_y + min(max(v, 0), J.crop_h - 1)) * J.src_stride);
                w[u] = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int      b  = ch * 4 + k;
                    const int      bo = sx0 + b;
                    const bool     ok = b < sb && vin && (!J.padded || (bo >= 0 && bo < rowb));
                    const uint32_t x  = row[min(max(bo, 0), rowb - 1)];
                    w[u] |= (ok ? x : 0u) << (8 * k);
                }
                at[u] = qv ? rr * SW + kSepPadL + ch * 4 : -1;
                r += dr, ch += dc;
                if (ch >= nch) ch -= nch, r++;
            }
#pragma unroll
            for (int u = 0; u < kBatch; u++)
                if (at[u] >= 0) *(uint32_t*)(S + at[u]) = w[u];
        }
    }
    __syncthreads();
    // staged row rr's first byte (column u_lo)
    const int  shift0 = J.padded ? 0 : (int)(rowa0 & 15), sstep = J.padded ? 0 : (int)(J.src_stride & 15);
    const auto srow   = [&](int rr) { return S + rr * SW + kSepPadL + ((shift0 + (r_lo + rr) * sstep) & 15); };
    // The replicated border: taps left of column 0 read column 0, right of crop_w - 1 read crop_w - 1
    // (the anchors are clamped into the crop, so at most K/2 - 1 and K/2 columns).
    // (INTER_AREA's taps stay inside the crop: its zero-weight padding taps read whatever follows)
    const int padl = AREA ? 0 : max(0, -(xt[0] - k2 + 1)), padr = AREA ? 0 : max(0, xt[(nx - 1) * xs] + k2 - (J.crop_w - 1));
    if (padl + padr > 0) { // (uniform; u_lo = 0 when padl, u_hi = crop_w - 1 when padr)
        const int per = (padl + padr) * cn;
        for (int i = tid; i < nr * per; i += nt) {
            const int rr = i / per, k = i - rr * per, p = k / cn, c = k - p * cn;
            uint8_t*  row = srow(rr);
            if (p < padl) row[-(p + 1) * cn + c] = row[c];
            else row[(J.crop_w - u_lo + (p - padl)) * cn + c] = row[(J.crop_w - 1 - u_lo) * cn + c];
        }
        __syncthreads();
    }
    // The lane's 4 elements: 4 consecutive bytes of the window row (a u8 window: one dword store),
    // or, for a final_out job, 4 consecutive pixels of one channel (one float4 store into its plane).
    const int nb = nx * cn, e0 = tid * 4;
    const int gpr = (nx + 3) >> 2, lc = tid / gpr, px0 = (tid - lc * gpr) * 4;
    const bool planar = J.final_out != 0;
    // (the host sizes bands so that every element has a lane; a band that outgrew the workgroup would
    // leave outputs unwritten: reported, never silent)
    if (tid == 0 && (planar ? cn * gpr : (nb + 3) >> 2) > nt) atomicOr(error, 512);
    if (planar ? lc >= cn : e0 >= nb) return; // (no barrier below; the LUT was published by the staging barrier)
    int px[4], ch[4], xe[4]; // pixel in the tile, channel, element of the full destination row
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = min(e0 + q, nb - 1);
        px[q]       = planar ? min(px0 + q, nx - 1) : e / cn;
        ch[q]       = planar ? lc : e - (e / cn) * cn;
        xe[q]       = (J.win_x + x0 + px[q]) * cn + ch[q];
    }
    // element q's first tap in a staged row (its taps: + j * cn), and the coefficients
    int ob[4], cf[4][K];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int  i = px[q], c = ch[q];
        const int* t = xt + i * xs;
        ob[q]        = (t[0] - k2 + 1 - u_lo) * cn + c;
#pragma unroll
        for (int j = 0; j < K; j++) cf[q][j] = AREA ? (j < t[1] ? t[2 + j] : 0) : t[1 + j]; // (area: float bits; +0.f)
    }
    const int W = J.dst_w * cn, xv = simd_end(K, W), xmax = max(max(xe[0], xe[1]), max(xe[2], xe[3]));
    // The window: hw[j][q] = horizontal sum of source row clamp(sy - K/2 + 1 + j) for element q (float
    // for the cubic vector form, exact: |sum| < 2^24; int otherwise).  The rows follow sy, which grows
    // with the output row, so a step of d rows keeps hw[d..K) as hw[0..K - d) and sums the d new rows:
    // d is workgroup-uniform (a scalar switch, register indices constant in every case).
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    using HT = typename std::conditional<K == 4 || AREA, float, int>::type;
    HT  hw[K][4] = {};
    int wsy      = 0;
    const auto hsum = [&](int j, int sy) {
        // (area: rows past the tile's last are its last, weighted 0)
        const int      rr  = AREA ? min(sy + j - r_lo, nr - 1) : min(max(sy - k2 + 1 + j, 0), J.crop_h - 1) - r_lo;
        const uint8_t* row = srow(rr);
        if constexpr (AREA) { // buf[dx] += S[sx] * alpha from 0, in tap order
            int b[4][K];
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int jj = 0; jj < K; jj++) b[q][jj] = row[ob[q] + jj * cn];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float acc = 0.f;
#pragma unroll
                for (int jj = 0; jj < K; jj++) acc = acc + (float)b[q][jj] * __int_as_float(cf[q][jj]);
                hw[j][q] = acc;
            }
            return;
        }
        // the row's taps read together, then the sums (the compiler would otherwise wait for each
        // element's reads before issuing the next element's) -- up to K = AEON_SEP_SCHED
        if constexpr (K <= AEON_SEP_SCHED) {
            int b[4][K];
#pragma unroll
            for (int q = 0; q < 4; q++)
#pragma unroll
                for (int jj = 0; jj < K; jj++) b[q][jj] = row[ob[q] + jj * cn];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int acc = 0;
#pragma unroll
                for (int jj = 0; jj < K; jj++) acc = mad_i24(b[q][jj], cf[q][jj], acc);
                hw[j][q] = (HT)((AEON_RG_SKIP & 1) ? rr + q : acc);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint8_t* e   = row + ob[q];
                int            acc = 0;
#pragma unroll
                for (int jj = 0; jj < K; jj++) acc = mad_i24((int)e[jj * cn], cf[q][jj], acc);
                hw[j][q] = (HT)((AEON_RG_SKIP & 1) ? rr + q : acc);
            }
        }
    };
    for (int r = 0; r < ny; r++) {
        const int* t  = yt + r * xs;
        const int  sy = __builtin_amdgcn_readfirstlane(t[0]);
        const int  d  = (r == 0 || sy < wsy || sy - wsy > K) ? K : sy - wsy;
        wsy           = sy;
        sep_shift<K>(d, [&](auto D) {
            constexpr int dd = decltype(D)::value;
#pragma unroll
            for (int j = 0; j + dd < K; j++)
#pragma unroll
                for (int q = 0; q < 4; q++) hw[j][q] = hw[j + dd][q];
#pragma unroll
            for (int j = K - dd; j < K; j++) hsum(j, sy);
        });
        int coef[K] = {};
        if constexpr (!AREA)
#pragma unroll
            for (int j = 0; j < K; j++) coef[j] = __builtin_amdgcn_readfirstlane(t[1 + j]);
        uint32_t word = 0;
        if constexpr (K == 4 && !AREA) { // VResizeCubicVec_32s8u, SSE's order of operations, two elements per packed op
            const float sc = 1.f / (2048 * 2048);
            const float c0 = (float)coef[0] * sc, c1 = (float)coef[1] * sc, c2 = (float)coef[2] * sc, c3 = (float)coef[3] * sc;
#pragma unroll
            for (int p2 = 0; p2 < 2; p2++) {
                const int qa = 2 * p2, qb = qa + 1;
                f32x2     sm = (f32x2){hw[0][qa], hw[0][qb]} * (f32x2){c0, c0} + (f32x2){hw[1][qa], hw[1][qb]} * (f32x2){c1, c1};
                sm           = sm + (f32x2){hw[2][qa], hw[2][qb]} * (f32x2){c2, c2};
                sm           = sm + (f32x2){hw[3][qa], hw[3][qb]} * (f32x2){c3, c3};
                // saturate_cast<uchar>(saturate_cast<short>(cvRound(s))): round half to even, clamp to
                // [0, 255], in one v_cvt_pk_u8_f32 per element
                word = __builtin_amdgcn_cvt_pk_u8_f32(sm.x, (uint32_t)qa, word);
                word = __builtin_amdgcn_cvt_pk_u8_f32(sm.y, (uint32_t)qb, word);
            }
        }
        if constexpr (AREA) { // sum = beta0 * h0, sum += beta_k * h_k; saturate_cast<uchar>(cvRound)
            const int n = __builtin_amdgcn_readfirstlane(t[1]);
            float     beta[K];
#pragma unroll
            for (int j = 0; j < K; j++) beta[j] = j < n ? __int_as_float(__builtin_amdgcn_readfirstlane(t[2 + j])) : 0.f;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float sum = beta[0] * hw[0][q];
#pragma unroll
                for (int j = 1; j < K; j++) sum = sum + beta[j] * hw[j][q];
                word |= (uint32_t)sat_u8((int)__builtin_rintf(sum)) << (8 * q);
            }
        } else if (K != 4 || xmax >= xv) { // the other forms, and elements on the scalar tail
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int x = xe[q];
                int       v;
                if (K == 4 && x < xv) continue;
                if (K == 2 && x < xv) { // VResizeLinearVec_32s8u
                    const int m = sat_s16(((sat_s16((int)hw[0][q] >> 4) * coef[0]) >> 16) +
                                          ((sat_s16((int)hw[1][q] >> 4) * coef[1]) >> 16));
                    v           = sat_u8(sat_s16(m + 2) >> 2);
                } else { // FixedPtCast<int, uchar, 22>, int32 sums wrapping
                    uint32_t acc = 0;
                    if constexpr (K == 4) {
#pragma unroll
                        for (int j = 0; j < K; j++) acc += (uint32_t)(int)hw[j][q] * (uint32_t)coef[j];
                    } else { // (|hw|, |coef| < 2^23: the 24-bit product's low 32 bits are the wrapping product)
#pragma unroll
                        for (int j = 0; j < K; j++) acc = (uint32_t)mad_i24((int)hw[j][q], coef[j], (int)acc);
                    }
                    v = sat_u8((int32_t)(acc + (1u << 21)) >> 22);
                }
                word = (word & ~(0xffu << (8 * q))) | ((uint32_t)v << (8 * q));
            }
        }
        if (planar) {
            if (!(AEON_RG_SKIP & 2) || word == 0x12345678u) store_planar(J, lut, bgr, chm, y0 + r, x0 + px0, lc, nx - px0, word);
            continue;
        }
        const auto dst = out + ((size_t)(y0 + r) * J.win_w + x0) * cn + e0;
        if ((AEON_RG_SKIP & 2) && word != 0x12345678u) {
        } else if (e0 + 4 <= nb && ((uintptr_t)dst & 3) == 0) {
            *(__attribute__((address_space(1))) uint32_t*)dst = word;
        } else {
            for (int q = 0; q < 4 && e0 + q < nb; q++) dst[q] = (uint8_t)(word >> (8 * q));
        }
    }
}

// The device half of interpolateLanczos4 (OpenCV 2.4.9 imgwarp.cpp; the host half: lanczos4_inputs,
// stage.cpp): per destination column / row the eight coefficients from the fraction f and the host's
// sin / cos of y0 -- the same IEEE float and double operations in the same order (no contraction:
// -ffp-contract=off; correctly rounded divisions) -- normalised to sum 1 in float, then the 11-bit
// fixed point of the taps.
__global__ __launch_bounds__(256) void lanczos4_taps(const LzIn* __restrict__ in, GrTap* __restrict__ out, int n)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const LzIn L = in[i];
    const double s45 = 0.70710678118654752440084436210485;
    const double cs0[8] = {1, -s45, 0, s45, -1, s45, 0, -s45}, cs1[8] = {0, -s45, 1, -s45, 0, s45, -1, s45};
    const double kPi = 3.1415926535897932384626433832795;
    float c[8];
    if (L.f < FLT_EPSILON) {
#pragma unroll
        for (int k = 0; k < 8; k++) c[k] = k == 3 ? 1.f : 0.f;
    } else {
        float sum = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const double y = -(L.f + 3 - k) * kPi * 0.25;
            c[k]           = (float)((cs0[k] * L.s0 + cs1[k] * L.c0) / (y * y));
            sum += c[k];
        }
        sum = __fdiv_rn(1.f, sum);
#pragma unroll
        for (int k = 0; k < 8; k++) c[k] *= sum;
    }
    GrTap t;
    t.s = L.s;
#pragma unroll
    for (int k = 0; k < 8; k++) t.c[k] = (int16_t)min(max((int)rintf(c[k] * 2048.f), -32768), 32767);
    out[i] = t;
}

hipError_t launch_lanczos4_taps(const LzIn* in, GrTap* out, int n, hipStream_t stream)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(lanczos4_taps, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, n);
    return hipGetLastError();
}

hipError_t launch_resize_sep(int K, bool area, const ResizeJob* jobs, const uint8_t* table, int n_jobs, int max_tiles, int TR,
                             int CW, int NR, int SW, int cn, const float* lut, int bgr, int chm, int32_t* error, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    const size_t lds = ((size_t)(CW + TR) * ((area ? 2 : 1) + K) * 4 + 15) / 16 * 16 + (size_t)NR * SW + (lut ? 768 * 4 : 0);
    const int    threads = std::min(256, (std::max((CW * cn + 3) / 4, cn * ((CW + 3) / 4)) + 63) / 64 * 64);
    const dim3   grid((unsigned)max_tiles, (unsigned)n_jobs);
    const bool c3 = cn == 3; // (every job of a resize_sep launch has the launch's channel count)
    typedef void (*SepFn)(const ResizeJob*, const uint8_t*, int, int, int, int, const float*, int, int, int32_t*);
    SepFn fn = nullptr;
    if (area) {
        if (K == 4) fn = c3 ? resize_sep<4, 3, true> : resize_sep<4, 0, true>;
        else if (K == 8) fn = c3 ? resize_sep<8, 3, true> : resize_sep<8, 0, true>;
        else return hipErrorInvalidValue;
    } else switch (K) {
    case 2: fn = c3 ? resize_sep<2, 3> : resize_sep<2, 0>; break;
    case 4: fn = c3 ? resize_sep<4, 3> : resize_sep<4, 0>; break;
    case 8: fn = c3 ? resize_sep<8, 3> : resize_sep<8, 0>; break;
    default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(fn, grid, dim3(threads), lds, stream, jobs, table, TR, CW, NR, SW, lut, bgr, chm, error);
    return hipGetLastError();
}

hipError_t launch_resize_generic(const ResizeJob* jobs, const uint8_t* table, int n_jobs, int max_tiles, int TR, int CW,
                                 int NR, int xs, int amax, int cn_max, int SW, const float* lut, int bgr, int chm,
                                 int32_t* error, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    const size_t lds = ((size_t)CW * xs + (size_t)TR * xs + (size_t)NR * CW * cn_max) * 4 + (size_t)NR * SW + (lut ? 768 * 4 : 0);
    hipLaunchKernelGGL(resize_generic, dim3((unsigned)max_tiles, (unsigned)n_jobs), dim3(256), lds, stream, jobs, table, TR,
                       CW, NR, xs, amax, SW, lut, bgr, chm, error);
    return hipGetLastError();
}

} // namespace aeon_hip
