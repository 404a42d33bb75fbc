// augment_kernels.hip -- CDNA4 (gfx950) kernels for aeon's per-record image path.
//
// One workgroup = one (image, band of output rows) tile.  The workgroup stages the source
// rows its band needs into LDS (coalesced 16-byte buffer loads of packed HWC uint8,
// re-laid as one 32-bit word per pixel), builds the per-column / per-row OpenCV resize
// coefficients in LDS, then each lane produces 4 consecutive output pixels:
//   resize (OpenCV 2.4 INTER_LINEAR fixed point incl. the SSE2 vertical formula, 2x area,
//   nearest or copy) -> brightness/saturation cv::transform -> hue (HSV8 round trip) ->
//   contrast -> lighting -> flip (output index) -> BGR->RGB + HWC->CHW + standardize
//   (per-channel LUT, bit-exact with aeon's f64-per-op arithmetic) -> coalesced stores.
// Contrast needs the mean of the post-hue image: a KM_STATS launch of the same kernel
// writes exact per-tile integer channel sums, which the KM_FINAL launch reduces.
// Integer work throughout; no MFMA (nothing here is a dense contraction).
//
// Build with -ffp-contract=off: the float/double expressions must round exactly as
// aeon's x86 SSE2 build does (no FMA contraction).
#include <hip/hip_runtime.h>

#include "aug_job.hpp"

namespace aeon_hip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float    f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int sat_u8(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int sat_s16(int v) { return min(max(v, -32768), 32767); }
__device__ __forceinline__ int rnd(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int byte_of(uint32_t p, int c) { return (p >> (8 * c)) & 0xff; }

// ---- resize coefficients (OpenCV 2.4 resizeGeneric_ / resizeNN) -----------------------------
struct XTap {
    int sx, sx2, a0, a1;
};

__device__ __forceinline__ XTap xcoef(const AugJob& J, int dx)
{
    XTap t;
    const int sw = J.crop_w;
    switch (J.mode) {
    case RESIZE_LINEAR: {
        float fx = (float)((dx + 0.5) * J.scale_x - 0.5);
        int   sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) fx = 0.f, sx = 0;
        if (sx + 1 >= sw) fx = 0.f, sx = sw - 1;
        t.sx  = sx;
        t.a0  = sat_s16(rnd((1.f - fx) * 2048.f));
        t.a1  = sat_s16(rnd(fx * 2048.f));
        t.sx2 = t.a1 == 0 ? sx : sx + 1;
        break;
    }
    case RESIZE_AREA2X:
        t.sx = 2 * dx, t.sx2 = 2 * dx + 1, t.a0 = t.a1 = 0;
        break;
    case RESIZE_NEAREST: {
        int sx = (int)floor(dx * J.scale_x);
        t.sx = t.sx2 = min(sx, sw - 1), t.a0 = t.a1 = 0;
        break;
    }
    default:
        t.sx = t.sx2 = dx, t.a0 = t.a1 = 0;
    }
    return t;
}

struct YTap {
    int r0, r1, b0, b1;
};

__device__ __forceinline__ YTap ycoef(const AugJob& J, int dy)
{
    YTap      t;
    const int sh = J.crop_h;
    switch (J.mode) {
    case RESIZE_LINEAR: {
        float fy = (float)((dy + 0.5) * J.scale_y - 0.5);
        int   sy = (int)floorf(fy);
        fy -= (float)sy;
        t.b0 = sat_s16(rnd((1.f - fy) * 2048.f));
        t.b1 = sat_s16(rnd(fy * 2048.f));
        t.r0 = min(max(sy, 0), sh - 1);
        t.r1 = min(max(sy + 1, 0), sh - 1);
        break;
    }
    case RESIZE_AREA2X:
        t.r0 = 2 * dy, t.r1 = 2 * dy + 1, t.b0 = t.b1 = 0;
        break;
    case RESIZE_NEAREST:
        t.r0 = t.r1 = min((int)floor(dy * J.scale_y), sh - 1), t.b0 = t.b1 = 0;
        break;
    default:
        t.r0 = t.r1 = dy, t.b0 = t.b1 = 0;
    }
    return t;
}

// ---- photometric stages (aeon src/image.cpp:336-406 over OpenCV 2.4) ------------------------
__device__ __forceinline__ void bs_apply(const AugJob& J, int& b, int& g, int& r)
{
    if (J.bs_kind == BS_DIAG) { // diagtransform_8u
        b = sat_u8(rnd(J.bsm[0] * (float)b + 0.f));
        g = sat_u8(rnd(J.bsm[4] * (float)g + 0.f));
        r = sat_u8(rnd(J.bsm[8] * (float)r + 0.f));
    } else if (J.bs_kind == BS_FIXPT) { // transform_8u, 10-bit fixed point
        const int* q  = J.bsq;
        int        t0 = (q[0] * b + q[1] * g + q[2] * r + 512) >> 10;
        int        t1 = (q[3] * b + q[4] * g + q[5] * r + 512) >> 10;
        int        t2 = (q[6] * b + q[7] * g + q[8] * r + 512) >> 10;
        b = sat_u8(t0), g = sat_u8(t1), r = sat_u8(t2);
    } else { // transform_<uchar,float>
        const float* m  = J.bsm;
        float        fb = (float)b, fg = (float)g, fr = (float)r;
        int          t0 = rnd(m[0] * fb + m[1] * fg + m[2] * fr + 0.f);
        int          t1 = rnd(m[3] * fb + m[4] * fg + m[5] * fr + 0.f);
        int          t2 = rnd(m[6] * fb + m[7] * fg + m[8] * fr + 0.f);
        b = sat_u8(t0), g = sat_u8(t1), r = sat_u8(t2);
    }
}

constexpr int pack_sectors(int s0, int s1, int s2, int s3, int s4, int s5)
{
    return s0 | (s1 << 2) | (s2 << 4) | (s3 << 6) | (s4 << 8) | (s5 << 10);
}
constexpr int kSectorB = pack_sectors(1, 1, 3, 0, 0, 2);
constexpr int kSectorG = pack_sectors(3, 0, 0, 2, 1, 1);
constexpr int kSectorR = pack_sectors(0, 2, 1, 1, 3, 0);

// cvtColor(BGR2HSV) [RGB2HSV_b], H = (H + hue) % 180 stored as uchar, cvtColor(HSV2BGR)
// [HSV2RGB_b over HSV2RGB_f].
__device__ __forceinline__ void hue_apply(const int32_t* sdiv, const int32_t* hdiv, int hue, int& b,
                                          int& g, int& r)
{
    int v = max(b, max(g, r)), vmin = min(b, min(g, r));
    int diff = v - vmin;
    int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    int s = (diff * sdiv[v] + (1 << 11)) >> 12;
    int h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
    h = (h * hdiv[diff] + (1 << 11)) >> 12;
    h += h < 0 ? 180 : 0;
    int H = sat_u8(h);
    H     = ((H + hue) % 180) & 0xff;

    float hf = (float)H, sf = (float)s * (1.f / 255), vf = (float)v * (1.f / 255);
    float bb, gg, rr;
    if (sf == 0.f) {
        bb = gg = rr = vf;
    } else {
        hf *= 6.f / 180.f;
        while (hf >= 6.f) hf -= 6.f; // h >= 0 always here
        int sector = (int)floorf(hf);
        hf -= (float)sector;
        if ((unsigned)sector >= 6u) sector = 0, hf = 0.f;
        float t0 = vf;
        float t1 = vf * (1.f - sf);
        float t2 = vf * (1.f - sf * hf);
        float t3 = vf * (1.f - sf * (1.f - hf));
        // sector_data = {{1,3,0},{1,0,2},{3,0,1},{0,2,1},{0,1,3},{2,1,0}}, 2 bits per sector
        const int ib = (kSectorB >> (2 * sector)) & 3;
        const int ig = (kSectorG >> (2 * sector)) & 3;
        const int ir = (kSectorR >> (2 * sector)) & 3;
        bb = ib == 0 ? t0 : ib == 1 ? t1 : ib == 2 ? t2 : t3;
        gg = ig == 0 ? t0 : ig == 1 ? t1 : ig == 2 ? t2 : t3;
        rr = ir == 0 ? t0 : ir == 1 ? t1 : ir == 2 ? t2 : t3;
    }
    b = sat_u8(rnd(bb * 255.f));
    g = sat_u8(rnd(gg * 255.f));
    r = sat_u8(rnd(rr * 255.f));
}

// ---- source staging ----------------------------------------------------------------------------
// Stage resize-source rows [v_lo, v_lo+nr) x cols [u_lo, u_lo+nc) as one 32-bit word per pixel.
__device__ __forceinline__ void stage_rows(const AugJob& J, uint32_t* stage, int pitch, int v_lo,
                                           int nr, int u_lo, int nc)
{
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)J.src_ptr, (short)0, (int)J.src_bytes, 0x00020000);
    const int cn     = J.cn;
    const int groups = (nc + 3) >> 2;
    const int total  = nr * groups;
    for (int w = threadIdx.x; w < total; w += kBlock) {
        const int j  = w / groups;
        const int g  = w - j * groups;
        const int v  = v_lo + j;
        const int u0 = u_lo + 4 * g;
        const int cy = v + J.shift_y;     // row inside the crop
        const int cx = u0 + J.shift_x;    // first column inside the crop
        uint32_t  px[4];
        const bool row_ok = cy >= 0 && cy < J.crop_h;
        if (row_ok && cx >= 0 && cx + 3 < J.crop_w) {
            const int b = (J.crop_y + cy) * J.src_stride + (J.crop_x + cx) * cn;
            const int a = b & ~3, sh = b & 3;
            if (cn == 3) {
                u32x4    d  = __builtin_amdgcn_raw_buffer_load_b128(rsrc, a, 0, 0);
                uint32_t e0 = __builtin_amdgcn_alignbyte(d.y, d.x, sh);
                uint32_t e1 = __builtin_amdgcn_alignbyte(d.z, d.y, sh);
                uint32_t e2 = __builtin_amdgcn_alignbyte(d.w, d.z, sh);
                px[0] = e0 & 0xffffff;
                px[1] = (e0 >> 24) | ((e1 & 0xffff) << 8);
                px[2] = (e1 >> 16) | ((e2 & 0xff) << 16);
                px[3] = e2 >> 8;
            } else {
                u32x2    d  = __builtin_amdgcn_raw_buffer_load_b64(rsrc, a, 0, 0);
                uint32_t e0 = __builtin_amdgcn_alignbyte(d.y, d.x, sh);
                px[0] = e0 & 0xff, px[1] = (e0 >> 8) & 0xff, px[2] = (e0 >> 16) & 0xff, px[3] = e0 >> 24;
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int x = cx + k;
                uint32_t  p = 0;
                if (row_ok && x >= 0 && x < J.crop_w) {
                    const int b = (J.crop_y + cy) * J.src_stride + (J.crop_x + x) * cn;
                    for (int c = 0; c < cn; c++)
                        p |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, b + c, 0, 0) << (8 * c);
                }
                px[k] = p;
            }
        }
        u32x4 q = {px[0], px[1], px[2], px[3]};
        *(u32x4*)(stage + j * pitch + 4 * g) = q;
    }
}

// ---- the tile kernel -----------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(kBlock) void augment_tiles(LaunchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const AugJob& J    = a.jobs[blockIdx.y];
    const int     tile = blockIdx.x;
    if (tile >= J.tiles) return;
    if (MODE == KM_STATS && J.stats_slot < 0) return;

    const int TR    = a.rows_per_tile;
    const int y0    = tile * TR;
    const int nrows = min(TR, J.win_h - y0);
    const int tid   = threadIdx.x;
    const int cn    = J.cn;

    const LdsLayout L     = lds_layout(a.max_win_w, TR, a.stage_rows, a.stage_pitch);
    int32_t*        sdiv  = (int32_t*)(smem + L.hsv);
    int32_t*        hdiv  = sdiv + 256;
    float*          lut   = (float*)(smem + L.lut);
    int4*           xt    = (int4*)(smem + L.xt);  // only .x/.y used (packed), 8 B per column
    int4*           yt    = (int4*)(smem + L.yt);
    int32_t*        red   = (int32_t*)(smem + L.red);
    double*         shift = (double*)(smem + L.red + 64);
    uint32_t*       stage = (uint32_t*)(smem + L.stage);
    const int       pitch = a.stage_pitch;

    // source window of this band (uniform; resize coefficients are monotone in dx, dy)
    const XTap xf = xcoef(J, J.win_x), xl = xcoef(J, J.win_x + J.win_w - 1);
    const YTap yf = ycoef(J, J.win_y + y0), yl = ycoef(J, J.win_y + y0 + nrows - 1);
    const int  u_lo = xf.sx;
    const int  u_hi = max(xl.sx2, xl.sx);
    const int  v_lo = yf.r0;
    const int  v_hi = max(yl.r1, yl.r0);
    const int nc = u_hi - u_lo + 1, nr = v_hi - v_lo + 1;
    if (nc > pitch || nr > a.stage_rows || J.win_w > a.max_win_w) {
        if (tid == 0) atomicOr(a.error, 1);
        return;
    }

    // per-column taps (relative to u_lo) and weights; flip is applied on the output index
    int2* xt2 = (int2*)xt;
    for (int x = tid; x < J.win_w; x += kBlock) {
        XTap t = xcoef(J, J.win_x + x);
        xt2[x] = make_int2((t.sx - u_lo) | ((t.sx2 - u_lo) << 16), (t.a0 & 0xffff) | (t.a1 << 16));
    }
    for (int r = tid; r < nrows; r += kBlock) {
        YTap t = ycoef(J, J.win_y + y0 + r);
        yt[r]  = make_int4((t.r0 - v_lo) * pitch, (t.r1 - v_lo) * pitch, t.b0, t.b1);
    }
    const bool do_photo = MODE != KM_RAW && cn == 3;
    const int  photo    = do_photo ? J.photo : 0;
    if (photo & PHOTO_HUE) {
        sdiv[tid] = a.hsv_tables[tid];
        hdiv[tid] = a.hsv_tables[256 + tid];
    }
    const bool use_lut = MODE == KM_FINAL && a.out_dtype == OUT_F32 && a.lut != nullptr;
    if (use_lut)
        for (int i = tid; i < 3 * 256; i += kBlock) lut[i] = a.lut[i];
    if (MODE == KM_FINAL && (photo & PHOTO_CONTRAST) && tid < 64) {
        // reduce the exact per-tile channel sums of this image (written by KM_STATS)
        unsigned long long s0 = 0, s1 = 0, s2 = 0;
        for (int t = tid; t < J.tiles; t += 64) {
            const uint32_t* p = a.partials + ((size_t)J.stats_slot * a.max_tiles + t) * 4;
            s0 += p[0], s1 += p[1], s2 += p[2];
        }
        for (int o = 32; o > 0; o >>= 1) {
            s0 += __shfl_xor(s0, o);
            s1 += __shfl_xor(s1, o);
            s2 += __shfl_xor(s2, o);
        }
        if (tid == 0) {
            // cv::mean = sum * (1./N); (1.0 - c) * mean, kept in f64
            const double inv_n = 1. / (double)(J.win_w * J.win_h);
            const double k     = 1.0 - (double)J.contrast;
            shift[0] = k * ((double)s0 * inv_n);
            shift[1] = k * ((double)s1 * inv_n);
            shift[2] = k * ((double)s2 * inv_n);
        }
    }
    stage_rows(J, stage, pitch, v_lo, nr, u_lo, nc);
    __syncthreads();

    const int gpr   = (J.win_w + 3) >> 2;
    const int total = nrows * gpr;
    uint32_t  sum0 = 0, sum1 = 0, sum2 = 0;
    double    sh0 = 0, sh1 = 0, sh2 = 0;
    if (MODE == KM_FINAL && (photo & PHOTO_CONTRAST)) sh0 = shift[0], sh1 = shift[1], sh2 = shift[2];

    uint8_t* out_item = (uint8_t*)J.out_ptr;
    const int plane   = J.win_w * J.win_h;

    for (int w = tid; w < total; w += kBlock) {
        const int  ry  = w / gpr;
        const int  cg  = w - ry * gpr;
        const int4 ytr = yt[ry];
        const int  y   = y0 + ry; // window row
        int        val[4][3];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int ox = cg * 4 + k;
            val[k][0] = val[k][1] = val[k][2] = 0;
            if (ox >= J.win_w) continue;
            const int  x   = J.flip ? J.win_w - 1 - ox : ox;
            const int2 xtt = xt2[x];
            const int  sx = xtt.x & 0xffff, sx2 = xtt.x >> 16;
            const uint32_t p00 = stage[ytr.x + sx], p01 = stage[ytr.x + sx2];
            int            v3[3] = {0, 0, 0};
            if (J.mode == RESIZE_LINEAR) {
                const uint32_t p10 = stage[ytr.y + sx], p11 = stage[ytr.y + sx2];
                const int      a0 = (short)(xtt.y & 0xffff), a1 = xtt.y >> 16;
                const int      e0 = (J.win_x + x) * cn;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    if (c >= cn) break;
                    const int H0 = byte_of(p00, c) * a0 + byte_of(p01, c) * a1;
                    const int H1 = byte_of(p10, c) * a0 + byte_of(p11, c) * a1;
                    int       v;
                    if (e0 + c < J.xv) { // VResizeLinearVec_32s8u (SSE2)
                        const int m = ((H0 >> 4) * ytr.z >> 16) + ((H1 >> 4) * ytr.w >> 16);
                        v = (m + 2) >> 2;
                    } else { // FixedPtCast<int, uchar, 22>
                        v = (H0 * ytr.z + H1 * ytr.w + (1 << 21)) >> 22;
                    }
                    v3[c] = sat_u8(v);
                }
            } else if (J.mode == RESIZE_AREA2X) {
                const uint32_t p10 = stage[ytr.y + sx], p11 = stage[ytr.y + sx2];
#pragma unroll
                for (int c = 0; c < 3; c++)
                    v3[c] = (byte_of(p00, c) + byte_of(p01, c) + byte_of(p10, c) + byte_of(p11, c) + 2) >> 2;
            } else {
#pragma unroll
                for (int c = 0; c < 3; c++) v3[c] = byte_of(p00, c);
            }
            int b = v3[0], g = v3[1], r = v3[2];
            if (photo & PHOTO_BS) bs_apply(J, b, g, r);
            if (photo & PHOTO_HUE) hue_apply(sdiv, hdiv, J.hue, b, g, r);
            if (MODE == KM_STATS) {
                sum0 += b, sum1 += g, sum2 += r;
                continue;
            }
            if (photo & PHOTO_CONTRAST) {
                const float c = J.contrast;
                b = sat_u8(rnd((float)((double)((float)b * c + 0.f) + sh0)));
                g = sat_u8(rnd((float)((double)((float)g * c + 0.f) + sh1)));
                r = sat_u8(rnd((float)((double)((float)r * c + 0.f) + sh2)));
            }
            if (photo & PHOTO_LIGHTING) {
                const float la = J.light_a;
                b = sat_u8(sat_u8(rnd((float)b * la + 0.f)) + J.light_add[0]);
                g = sat_u8(sat_u8(rnd((float)g * la + 0.f)) + J.light_add[1]);
                r = sat_u8(sat_u8(rnd((float)r * la + 0.f)) + J.light_add[2]);
            }
            val[k][0] = b, val[k][1] = g, val[k][2] = r;
        }
        if (MODE == KM_STATS) continue;

        const int ox0 = cg * 4;
        const int nk  = min(4, J.win_w - ox0);
        if (MODE == KM_RAW) { // HWC uint8, source channel order
            uint8_t* d = out_item + ((size_t)y * J.win_w + ox0) * cn;
#pragma unroll
            for (int k = 0; k < 4; k++)
#pragma unroll
                for (int c = 0; c < 3; c++)
                    if (k < nk && c < cn) d[k * cn + c] = (uint8_t)val[k][c];
            continue;
        }
        // image::loader::load -- from_to {0,2,1,1,2,0} when bgr_to_rgb (a 3-channel config)
        if (a.bgr_to_rgb) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int t = val[k][0];
                val[k][0]   = val[k][2];
                val[k][2]   = t;
            }
        }
        if (a.channel_major) {
#pragma unroll
            for (int oc = 0; oc < 3; oc++) {
                if (oc >= cn) break;
                const size_t idx = (size_t)oc * plane + (size_t)y * J.win_w + ox0;
                if (a.out_dtype == OUT_F32) {
                    float f[4];
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        f[k] = use_lut ? lut[oc * 256 + val[k][oc]] : (float)val[k][oc];
                    float* d = (float*)out_item + idx;
                    if (a.vec_ok) {
                        f32x4 q = {f[0], f[1], f[2], f[3]};
                        __builtin_nontemporal_store(q, (f32x4*)d);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if (k < nk) d[k] = f[k];
                    }
                } else {
                    uint8_t* d = out_item + idx;
                    if (a.vec_ok) {
                        *(uint32_t*)d = val[0][oc] | (val[1][oc] << 8) | (val[2][oc] << 16) |
                                        ((uint32_t)val[3][oc] << 24);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            if (k < nk) d[k] = (uint8_t)val[k][oc];
                    }
                }
            }
        } else {
            const size_t base = ((size_t)y * J.win_w + ox0) * cn;
#pragma unroll
            for (int k = 0; k < 4; k++)
#pragma unroll
                for (int oc = 0; oc < 3; oc++) {
                    if (k >= nk || oc >= cn) continue;
                    if (a.out_dtype == OUT_F32)
                        ((float*)out_item)[base + k * cn + oc] =
                            use_lut ? lut[oc * 256 + val[k][oc]] : (float)val[k][oc];
                    else
                        out_item[base + k * cn + oc] = (uint8_t)val[k][oc];
                }
        }
    }

    if (MODE == KM_STATS) {
        for (int o = 32; o > 0; o >>= 1) {
            sum0 += __shfl_xor(sum0, o);
            sum1 += __shfl_xor(sum1, o);
            sum2 += __shfl_xor(sum2, o);
        }
        const int wave = tid >> 6, lane = tid & 63;
        if (lane == 0) red[wave * 4 + 0] = sum0, red[wave * 4 + 1] = sum1, red[wave * 4 + 2] = sum2;
        __syncthreads();
        if (tid < 3) {
            uint32_t s = 0;
            for (int wv = 0; wv < kBlock / 64; wv++) s += (uint32_t)red[wv * 4 + tid];
            a.partials[((size_t)J.stats_slot * a.max_tiles + tile) * 4 + tid] = s;
        }
    }
}

template __global__ void augment_tiles<KM_FINAL>(LaunchArgs);
template __global__ void augment_tiles<KM_STATS>(LaunchArgs);
template __global__ void augment_tiles<KM_RAW>(LaunchArgs);

// Host-side launch helpers (called from plan.cpp / capi.cpp).
hipError_t launch_tiles(int mode, const LaunchArgs& a, int n_jobs, hipStream_t stream)
{
    dim3 grid(a.max_tiles, n_jobs), block(kBlock);
    switch (mode) {
    case KM_FINAL:
        hipLaunchKernelGGL(augment_tiles<KM_FINAL>, grid, block, a.lds_bytes, stream, a);
        break;
    case KM_STATS:
        hipLaunchKernelGGL(augment_tiles<KM_STATS>, grid, block, a.lds_bytes, stream, a);
        break;
    default:
        hipLaunchKernelGGL(augment_tiles<KM_RAW>, grid, block, a.lds_bytes, stream, a);
    }
    return hipGetLastError();
}

hipError_t set_kernel_lds_limit(int bytes)
{
    hipError_t e;
    if ((e = hipFuncSetAttribute((const void*)augment_tiles<KM_FINAL>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, bytes)) != hipSuccess)
        return e;
    if ((e = hipFuncSetAttribute((const void*)augment_tiles<KM_STATS>,
                                 hipFuncAttributeMaxDynamicSharedMemorySize, bytes)) != hipSuccess)
        return e;
    return hipFuncSetAttribute((const void*)augment_tiles<KM_RAW>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

} // namespace aeon_hip
