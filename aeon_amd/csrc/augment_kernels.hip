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

// Minimum waves per SIMD the register allocator must leave room for (__launch_bounds__).
#ifndef AEON_HIP_MIN_WAVES
#define AEON_HIP_MIN_WAVES 1
#endif

namespace aeon_hip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float    f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));

__device__ __forceinline__ int sat_u8(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int sat_s16(int v) { return min(max(v, -32768), 32767); }
__device__ __forceinline__ int rnd(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int byte_of(uint32_t p, int c) { return (p >> (8 * c)) & 0xff; }
// 16x16-bit signed product (v_mul_i32_i24 with word selects): both operands must fit int16
__device__ __forceinline__ int mul16(int a, int b) { return (int)(short)a * (int)(short)b; }

// LDS accesses by byte address.  The kernel has no static LDS, so the dynamic area starts at
// LDS address 0 (checked at kernel entry); addressing through local-address-space pointers made
// from byte offsets lets the compiler fold constant parts into the ds_read offset field instead
// of adding the dynamic area's base at run time.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) float    lds_f32;
__device__ __forceinline__ uint32_t lds_ld(int byte_addr) { return *(const lds_u32*)(size_t)(uint32_t)byte_addr; }
__device__ __forceinline__ float    lds_ldf(int byte_addr) { return *(const lds_f32*)(size_t)(uint32_t)byte_addr; }

// ---- resize coefficients (OpenCV 2.4 resizeGeneric_ / resizeNN) -----------------------------
// Taps are (sx, sx+1) and (r0, r1); a weight of 0 marks a single-tap column / row.
struct XTap {
    int sx, a0, a1;
};

template <int RM>
__device__ __forceinline__ XTap xcoef(int dx, double scale, int sw)
{
    XTap t;
    if (RM == RESIZE_LINEAR) {
        float fx = (float)((dx + 0.5) * scale - 0.5);
        int   sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) fx = 0.f, sx = 0;
        if (sx + 1 >= sw) fx = 0.f, sx = sw - 1;
        t.sx = sx;
        t.a0 = sat_s16(rnd((1.f - fx) * 2048.f));
        t.a1 = sat_s16(rnd(fx * 2048.f));
    } else if (RM == RESIZE_AREA2X) {
        t.sx = 2 * dx, t.a0 = t.a1 = 0;
    } else if (RM == RESIZE_NEAREST) {
        t.sx = min((int)floor(dx * scale), sw - 1), t.a0 = t.a1 = 0;
    } else {
        t.sx = dx, t.a0 = t.a1 = 0;
    }
    return t;
}

struct YTap {
    int r0, r1, b0, b1;
};

template <int RM>
__device__ __forceinline__ YTap ycoef(int dy, double scale, int sh)
{
    YTap t;
    if (RM == RESIZE_LINEAR) {
        float fy = (float)((dy + 0.5) * scale - 0.5);
        int   sy = (int)floorf(fy);
        fy -= (float)sy;
        t.b0 = sat_s16(rnd((1.f - fy) * 2048.f));
        t.b1 = sat_s16(rnd(fy * 2048.f));
        t.r0 = min(max(sy, 0), sh - 1);
        t.r1 = min(max(sy + 1, 0), sh - 1);
    } else if (RM == RESIZE_AREA2X) {
        t.r0 = 2 * dy, t.r1 = 2 * dy + 1, t.b0 = t.b1 = 0;
    } else if (RM == RESIZE_NEAREST) {
        t.r0 = t.r1 = min((int)floor(dy * scale), sh - 1), t.b0 = t.b1 = 0;
    } else {
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
// A band stages resize-source rows [v_lo, v_lo+nr) x cols [u_lo, u_lo+nc) into LDS as one 32-bit
// word per pixel.  Items are 4-pixel groups; lane t takes items t, t+nt, ... in batches of
// kPrefetch whose loads are all in flight before the first is unpacked.  Each item is ONE load
// at its exact byte offset (12 bytes for 3 channels, 4 for 1 -- dword-unaligned buffer loads
// return the exact bytes on gfx950), unpacked with two v_perm, and written with one ds_write_b128.
// The walk over items keeps byte offsets incrementally: no 32-bit multiplies per item.
constexpr int kPrefetch = 4;

struct StageGeom {
    int v_lo, nr, u_lo, nc, groups;
};

struct Walk { // lane-private position of its next item
    int j, g; // staged row / 4-pixel group
    int src;  // source byte offset of the group's first pixel
    int lds;  // LDS byte address of the item
};

struct WalkStep { // uniform: advancing by nt items
    int dj, dg, dsrc, dlds, wrap_src, wrap_lds;
};

struct Prefetch {
    u32x3    d[kPrefetch];
    uint32_t lds[kPrefetch]; // LDS byte address | 2 (item) | 1 (fast); 0 = no item
};

__device__ __forceinline__ void walk_init(const AugJob& J, const StageGeom& G, int i, int pitch, int stage_base,
                                          int nt, Walk& w, WalkStep& st)
{
    w.j   = i / G.groups;
    w.g   = i - w.j * G.groups;
    w.src = (J.crop_y + G.v_lo + J.shift_y + w.j) * J.src_stride + (J.crop_x + G.u_lo + J.shift_x + 4 * w.g) * J.cn;
    w.lds = stage_base + (w.j * pitch + 4 * w.g) * 4;
    st.dj       = nt / G.groups;
    st.dg       = nt - st.dj * G.groups;
    st.dsrc     = st.dj * J.src_stride + st.dg * 4 * J.cn;
    st.dlds     = (st.dj * pitch + 4 * st.dg) * 4;
    st.wrap_src = J.src_stride - G.groups * 4 * J.cn;
    st.wrap_lds = (pitch - 4 * G.groups) * 4;
}

__device__ __forceinline__ void walk_next(const StageGeom& G, const WalkStep& st, Walk& w)
{
    w.j += st.dj, w.g += st.dg, w.src += st.dsrc, w.lds += st.dlds;
    if (w.g >= G.groups) w.g -= G.groups, w.j++, w.src += st.wrap_src, w.lds += st.wrap_lds;
}

// Fast item: the load lies wholly inside the image buffer (a buffer load that crosses num_records
// returns 0 for the whole access) and, for a padded job, inside the crop (outside it add_padding's
// zero border applies).  Unpadded, pixels right of the crop only ever meet a zero resize weight.
__device__ __forceinline__ bool stage_fast(const AugJob& J, const StageGeom& G, const Walk& w)
{
    const bool inside = (uint32_t)w.src + (J.cn == 3 ? 12u : 4u) <= (uint32_t)J.src_bytes;
    if (!J.padded) return inside;
    const int cy = G.v_lo + w.j + J.shift_y, cx = G.u_lo + 4 * w.g + J.shift_x;
    return inside && w.src >= 0 && cy >= 0 && cy < J.crop_h && cx >= 0 && cx + 3 < J.crop_w;
}

__device__ __forceinline__ u32x3 stage_load(const AugJob& J, __amdgpu_buffer_rsrc_t rsrc, int b)
{
    if (J.cn == 3) return __builtin_amdgcn_raw_buffer_load_b96(rsrc, b, 0, 0);
    return (u32x3){__builtin_amdgcn_raw_buffer_load_b32(rsrc, b, 0, 0), 0u, 0u};
}

__device__ __forceinline__ u32x4 stage_unpack(int cn, u32x3 d)
{
    if (cn == 3) // 12 bytes BGR BGR BGR BGR -> four (B, G, R, 0) words
        return (u32x4){d.x & 0xffffffu, __builtin_amdgcn_perm(d.y, d.x, 0x0C050403u),
                       __builtin_amdgcn_perm(d.z, d.y, 0x0C040302u), d.z >> 8};
    return (u32x4){d.x & 0xffu, __builtin_amdgcn_perm(0u, d.x, 0x0C0C0C01u), __builtin_amdgcn_perm(0u, d.x, 0x0C0C0C02u),
                   d.x >> 24};
}

// Slow item (add_padding border / crop edge of a padded job / buffer end): per-pixel byte loads,
// 0 outside the crop.
__device__ __forceinline__ u32x4 stage_slow(const AugJob& J, __amdgpu_buffer_rsrc_t rsrc, int cy, int cx)
{
    uint32_t   px[4];
    const bool row_ok = cy >= 0 && cy < J.crop_h;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = cx + k;
        uint32_t  p = 0;
        if (row_ok && x >= 0 && x < J.crop_w) {
            const int b = (J.crop_y + cy) * J.src_stride + (J.crop_x + x) * J.cn;
            for (int c = 0; c < J.cn; c++)
                p |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, b + c, 0, 0) << (8 * c);
        }
        px[k] = p;
    }
    return (u32x4){px[0], px[1], px[2], px[3]};
}

// Issue the loads of this lane's next kPrefetch items (fast items only) and advance the walk.
__device__ __forceinline__ void stage_issue(const AugJob& J, __amdgpu_buffer_rsrc_t rsrc, const StageGeom& G,
                                            const WalkStep& st, Walk& w, Prefetch& pf)
{
#pragma unroll
    for (int k = 0; k < kPrefetch; k++) {
        pf.lds[k] = 0;
        if (w.j < G.nr) {
            const bool fast = stage_fast(J, G, w);
            pf.lds[k]       = (uint32_t)w.lds | (fast ? 1u : 0u) | 2u;
            if (fast) pf.d[k] = stage_load(J, rsrc, w.src);
            walk_next(G, st, w);
        }
    }
}

// Unpack / load-slow and write this batch's items to LDS.
__device__ __forceinline__ void stage_commit(const AugJob& J, __amdgpu_buffer_rsrc_t rsrc, const StageGeom& G,
                                             const Prefetch& pf, int stage_base, int pitch)
{
#pragma unroll
    for (int k = 0; k < kPrefetch; k++) {
        const uint32_t m = pf.lds[k];
        if (!(m & 2)) continue;
        u32x4 q;
        if (m & 1) {
            q = stage_unpack(J.cn, pf.d[k]);
        } else { // rare: recover (row, group) from the LDS address
            const int o = (int)(m & ~3u) - stage_base;
            const int j = o / (pitch * 4), g = (o - j * pitch * 4) >> 4;
            q           = stage_slow(J, rsrc, G.v_lo + j + J.shift_y, G.u_lo + 4 * g + J.shift_x);
        }
        *(__attribute__((address_space(3))) u32x4*)(size_t)(m & ~3u) = q;
    }
}

// Stage a whole band: first batch already issued by the caller (pf, w), the rest here.
__device__ __forceinline__ void stage_finish(const AugJob& J, __amdgpu_buffer_rsrc_t rsrc, const StageGeom& G,
                                             const WalkStep& st, Walk& w, Prefetch& pf, int stage_base, int pitch)
{
    stage_commit(J, rsrc, G, pf, stage_base, pitch);
    while (w.j < G.nr) {
        stage_issue(J, rsrc, G, st, w, pf);
        stage_commit(J, rsrc, G, pf, stage_base, pitch);
    }
}

// Output cache policy: streaming stores (written once, read by the consumer of the batch).
#ifndef AEON_HIP_STORE_AUX
#define AEON_HIP_STORE_AUX 2 // nt
#endif
constexpr int kStoreAux = AEON_HIP_STORE_AUX;

__device__ __forceinline__ void store_f32x4(__amdgpu_buffer_rsrc_t r, int off, float a, float b, float c,
                                            float d)
{
    u32x4 v = {__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kStoreAux);
}

// One output pixel of the resize: 3 channels from the staged source (LDS).
// ytr = (row-0, row-1 LDS byte addresses in the staged band, b0, b1); col = byte offset of the
// first tap's column; wx = a0 | a1 << 16.  SCALED results are 4x the pixel value plus 0..3: the
// standardize LUT is addressed by (s & ~3) with no further shifts, and s >> 2 is the pixel.
// (Photometric kernels take plain values.)
template <int RM, bool SCALED>
__device__ __forceinline__ void resize_px(int4 ytr, int col, uint32_t wx, int s[3])
{
    const int a0 = ytr.x + col;
    if (RM == RESIZE_LINEAR) {
        const int      a1  = ytr.y + col;
        const uint32_t p00 = lds_ld(a0), p01 = lds_ld(a0 + 4), p10 = lds_ld(a1), p11 = lds_ld(a1 + 4);
        const u16x2     w   = __builtin_bit_cast(u16x2, wx); // (a0, a1)
#pragma unroll
        for (int c = 0; c < 3; c++) {
            // HResizeLinear: H = S[sx]*a0 + S[sx+1]*a1 (exact), one v_dot2_u32_u16 per row on
            // the (S[sx], S[sx+1]) byte pair that v_perm_b32 gathers into two u16 lanes.
            const uint32_t sel = (uint32_t)c | (0x0Cu << 8) | ((4u + c) << 16) | (0x0Cu << 24);
            const uint32_t H0  = __builtin_amdgcn_udot2(
                __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p01, p00, sel)), w, 0u, false);
            const uint32_t H1  = __builtin_amdgcn_udot2(
                __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p11, p10, sel)), w, 0u, false);
            // VResizeLinearVec_32s8u (SSE2): ((H0>>4)*b0 >> 16) + ((H1>>4)*b1 >> 16) + 2 >> 2.
            // The +2 rides in the high half of t0; the sum is <= 1023, so no saturation.
            const uint32_t t0 = (uint32_t)__mul24((int)(H0 >> 4), ytr.z) + (2u << 16);
            const uint32_t t1 = (uint32_t)__mul24((int)(H1 >> 4), ytr.w);
            s[c]              = (int)((t0 >> 16) + (t1 >> 16));
            if (!SCALED) s[c] >>= 2;
        }
    } else if (RM == RESIZE_AREA2X) {
        const int      a1  = ytr.y + col;
        const uint32_t p00 = lds_ld(a0), p01 = lds_ld(a0 + 4), p10 = lds_ld(a1), p11 = lds_ld(a1 + 4);
        // INTER_AREA 2x fast path: (a + b + c + d + 2) >> 2 per channel; channels 0/2 and 1
        // summed in 16-bit lanes (each sum <= 1022)
        const uint32_t m  = 0x00ff00ffu;
        const uint32_t lo = (p00 & m) + (p01 & m) + (p10 & m) + (p11 & m);
        const uint32_t hi = ((p00 >> 8) & m) + ((p01 >> 8) & m) + ((p10 >> 8) & m) + ((p11 >> 8) & m);
        s[0] = (int)(lo & 0xffff) + 2;
        s[1] = (int)(hi & 0xffff) + 2;
        s[2] = (int)(lo >> 16) + 2;
        if (!SCALED) s[0] >>= 2, s[1] >>= 2, s[2] >>= 2;
    } else {
        const uint32_t p00 = lds_ld(a0);
#pragma unroll
        for (int c = 0; c < 3; c++) s[c] = byte_of(p00, c) << (SCALED ? 2 : 0);
    }
}

// Elements of OpenCV's scalar row tail (e >= xv) use FixedPtCast<int, uchar, 22> instead.
template <bool SCALED>
__device__ __forceinline__ void tail_fix(int4 ytr, int col, uint32_t wx, int e0, int xv, int s[3])
{
    const uint32_t p00 = lds_ld(ytr.x + col), p01 = lds_ld(ytr.x + col + 4);
    const uint32_t p10 = lds_ld(ytr.y + col), p11 = lds_ld(ytr.y + col + 4);
    const int      a0 = wx & 0xffff, a1 = (int)(wx >> 16);
    for (int c = 0; c < 3; c++) {
        if (e0 + c < xv) continue;
        const int H0 = byte_of(p00, c) * a0 + byte_of(p01, c) * a1;
        const int H1 = byte_of(p10, c) * a0 + byte_of(p11, c) * a1;
        s[c]         = sat_u8((H0 * ytr.z + H1 * ytr.w + (1 << 21)) >> 22) << (SCALED ? 2 : 0);
    }
}

// standardize LUT (LDS offset 0) entry for source channel c at scaled value s
__device__ __forceinline__ float lut_at(int c, int s) { return lds_ldf(c * 1024 + (s & ~3)); }

enum OutForm : int { OF_F32_CHW_VEC = 0, OF_GENERIC = 1 };

// ---- the tile kernel -----------------------------------------------------------------------
// One workgroup = one chunk of rows_per_chunk output rows of one job, processed in bands of
// rows_per_tile rows through double-buffered LDS.
// KM: KM_FINAL (full record -> loader output), KM_STATS (contrast sums only), KM_RAW (resize
// only, HWC uint8: the resize_short pre-pass).  RM: ResizeMode of every job in the launch.
// PHOTO: the launch's jobs carry photometric work.  OF: output form (OF_F32_CHW_VEC = float32
// CHW planes, win_w % 4 == 0, 16-byte aligned items: the ImageNet configuration).
// TAIL: some LINEAR job of the launch has OpenCV scalar-tail columns (3*dst_w not covered by the
// SIMD loops); kept out of the common kernels, whose registers it would otherwise inflate.
template <int KM, int RM, bool PHOTO, int OF, bool TAIL>
__global__ __launch_bounds__(kBlockMax, AEON_HIP_MIN_WAVES) void augment_tiles(LaunchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem != 0u) { // see lds_ld
        if (threadIdx.x == 0) atomicOr(a.error, 4);
        return;
    }
    // The job descriptor is copied to registers before any store: the pixel loop then issues
    // no global loads except the next band's staging, so stores rarely make a load wait.
    const AugJob J     = a.jobs[blockIdx.y];
    const int    chunk = blockIdx.x;
    if (chunk >= J.tiles) return;
    if (KM == KM_STATS && J.stats_slot < 0) return;

    const int TR    = a.rows_per_tile;
    const int c0    = chunk * a.rows_per_chunk;
    const int c1    = min(c0 + a.rows_per_chunk, J.win_h);
    const int tid   = threadIdx.x;
    const int nt    = blockDim.x;
    const int cn    = J.cn;
    const int win_w = J.win_w;

    const LdsLayout L     = lds_layout(a.max_win_w, TR, a.stage_rows, a.stage_pitch, PHOTO && a.has_hue);
    float*          lut   = (float*)(smem + L.lut); // offset 0: immediate-offset reads per channel
    int32_t*        sdiv  = (int32_t*)(smem + L.hsv);
    int32_t*        hdiv  = sdiv + 256;
    int2*           xt    = (int2*)(smem + L.xt);
    int4*           yt0   = (int4*)(smem + L.yt);
    int32_t*        red   = (int32_t*)(smem + L.red);
    double*         shift = (double*)(smem + L.red + 128);
    const int       pitch = a.stage_pitch;

    // source columns (the same for every band; taps are monotone in dx)
    const XTap xf = xcoef<RM>(J.win_x, J.scale_x, J.crop_w);
    const XTap xl = xcoef<RM>(J.win_x + win_w - 1, J.scale_x, J.crop_w);
    const int  two_tap = (RM == RESIZE_LINEAR || RM == RESIZE_AREA2X) ? 1 : 0;
    StageGeom  G;
    G.u_lo   = xf.sx;
    G.nc     = xl.sx + two_tap - G.u_lo + 1;
    G.groups = (G.nc + 3) >> 2;
    if (G.nc > pitch || win_w > a.max_win_w) {
        if (tid == 0) atomicOr(a.error, 1);
        return;
    }
    auto band_rows = [&](int y0, StageGeom& g) { // rows of the band starting at window row y0
        const int n = min(TR, c1 - y0);
        g.v_lo      = ycoef<RM>(J.win_y + y0, J.scale_y, J.crop_h).r0;
        g.nr        = ycoef<RM>(J.win_y + y0 + n - 1, J.scale_y, J.crop_h).r1 - g.v_lo + 1;
        return n;
    };
    auto build_yt = [&](int y0, int n, const StageGeom& g, int4* yt) {
        for (int r = tid; r < n; r += nt) {
            const YTap t = ycoef<RM>(J.win_y + y0 + r, J.scale_y, J.crop_h);
            yt[r]        = make_int4(L.stage + (t.r0 - g.v_lo) * pitch * 4, L.stage + (t.r1 - g.v_lo) * pitch * 4,
                                     t.b0, t.b1);
        }
    };

    const __amdgpu_buffer_rsrc_t srsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)J.src_ptr, (short)0, (int)J.src_bytes, 0x00020000);
    // band 0 loads go out first; the tables below are built while they are in flight
    Prefetch pf;
    Walk     wk;
    WalkStep ws;
    int      n0 = band_rows(c0, G);
    if (G.nr > a.stage_rows) {
        if (tid == 0) atomicOr(a.error, 2);
        return;
    }
    walk_init(J, G, tid, pitch, L.stage, nt, wk, ws);
    stage_issue(J, srsrc, G, ws, wk, pf);

    for (int x = tid; x < win_w; x += nt) {
        const XTap t = xcoef<RM>(J.win_x + x, J.scale_x, J.crop_w);
        xt[x]        = make_int2(t.sx - G.u_lo, (t.a0 & 0xffff) | (t.a1 << 16));
    }
    const int photo = (PHOTO && KM != KM_RAW && cn == 3) ? J.photo : 0;
    if (photo & PHOTO_HUE)
        for (int i = tid; i < 512; i += nt) sdiv[i] = a.hsv_tables[i];
    const bool use_lut = KM == KM_FINAL && a.out_dtype == OUT_F32 && a.lut != nullptr;
    if (use_lut)
        for (int i = tid; i < 3 * 256; i += nt) lut[i] = a.lut[i];
    if (KM == KM_FINAL && (photo & PHOTO_CONTRAST) && tid < 64) {
        // reduce the exact per-chunk channel sums of this image (written by KM_STATS)
        unsigned long long s0 = 0, s1 = 0, s2 = 0;
        for (int t = tid; t < J.stats_tiles; t += 64) {
            const uint32_t* p = a.partials + ((size_t)J.stats_slot * a.partial_stride + t) * 4;
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
    build_yt(c0, n0, G, yt0);
    stage_finish(J, srsrc, G, ws, wk, pf, L.stage, pitch);
    __syncthreads();

    uint32_t sum0 = 0, sum1 = 0, sum2 = 0;
    double   sh0 = 0, sh1 = 0, sh2 = 0;
    if (KM == KM_FINAL && (photo & PHOTO_CONTRAST)) sh0 = shift[0], sh1 = shift[1], sh2 = shift[2];

    const int  elem  = (KM != KM_FINAL || a.out_dtype == OUT_U8) ? 1 : 4;
    const int  plane = win_w * J.win_h;
    const auto orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)J.out_ptr, (short)0,
                                                         plane * cn * elem, 0x00020000);
    const bool tail  = TAIL && RM == RESIZE_LINEAR && J.xv < J.dst_w * cn; // OpenCV scalar row tail
    const int  wx0   = J.win_x;
    const int  xv    = J.xv;
    const int  flip  = J.flip;
    const int  bgr   = a.bgr_to_rgb && cn == 3;
    // Lane -> (column group, row phase), fixed for the chunk: a lane's four output columns and
    // their taps stay in registers while it walks the band's rows.
    const int  gpr    = (win_w + 3) >> 2;
    const int  ncg    = min(gpr, nt);
    const int  nph    = nt / ncg;
    const int  lph    = tid / ncg;
    const int  lcg    = tid - lph * ncg;
    const bool active = lph < nph;
    // values carried from the resize to the store: 4x scaled (see resize_px) unless photometric
    constexpr bool SC = !PHOTO;
    auto lut_of       = [&](int c, int v) { return lut_at(c, SC ? v : v << 2); };
    auto u8_of        = [&](int v) { return SC ? v >> 2 : v; };

    int buf = 0;
    for (int y0 = c0; y0 < c1; y0 += TR) {
        const int   nrows = min(TR, c1 - y0);
        const int4* yt    = yt0 + buf * TR;
        const bool has_next = y0 + TR < c1;

        for (int cg = active ? lcg : gpr; cg < gpr; cg += ncg) {
            const int ox0 = cg * 4;
            const int nk  = min(4, win_w - ox0);
            int       col[4];
            uint32_t  wxk[4];
            int       tmask = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                // columns past the window edge recompute the last one (never stored)
                const int  ox  = min(ox0 + k, win_w - 1);
                const int  x   = flip ? win_w - 1 - ox : ox;
                const int2 xtt = xt[x];
                col[k]         = xtt.x * 4; // byte offset in a staged row
                wxk[k]         = (uint32_t)xtt.y;
                if (TAIL && RM == RESIZE_LINEAR && tail && (wx0 + x) * cn + 2 >= xv) tmask |= 1 << k;
            }
            for (int ry = lph; ry < nrows; ry += nph) {
                const int4 ytr = yt[ry];
                const int  y   = y0 + ry; // window row
                int        val[4][3];
#pragma unroll
                for (int k = 0; k < 4; k++) resize_px<RM, SC>(ytr, col[k], wxk[k], val[k]);
                if (TAIL && RM == RESIZE_LINEAR && tmask) {
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        if (tmask & (1 << k)) {
                            const int ox = min(ox0 + k, win_w - 1);
                            const int x  = flip ? win_w - 1 - ox : ox;
                            tail_fix<SC>(ytr, col[k], wxk[k], (wx0 + x) * cn, xv, val[k]);
                        }
                }
                if (PHOTO && photo) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        int b = val[k][0], g = val[k][1], r = val[k][2];
                        if (photo & PHOTO_BS) bs_apply(J, b, g, r);
                        if (photo & PHOTO_HUE) hue_apply(sdiv, hdiv, J.hue, b, g, r);
                        if (KM == KM_STATS) { // the intermediate keeps the post-hue pixel
                            if (k < nk) sum0 += b, sum1 += g, sum2 += r;
                            val[k][0] = b, val[k][1] = g, val[k][2] = r;
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
                        __builtin_amdgcn_sched_barrier(0); // one pixel's chain live at a time
                    }
                }
                if ((KM == KM_RAW || KM == KM_STATS) && cn == 3 && nk == 4) {
                    // HWC uint8, source channel order: 4 pixels = 12 bytes = one dwordx3 store
                    int v[4][3];
#pragma unroll
                    for (int k = 0; k < 4; k++)
#pragma unroll
                        for (int c = 0; c < 3; c++) v[k][c] = u8_of(val[k][c]);
                    const uint32_t w0 = v[0][0] | (v[0][1] << 8) | (v[0][2] << 16) | ((uint32_t)v[1][0] << 24);
                    const uint32_t w1 = v[1][1] | (v[1][2] << 8) | (v[2][0] << 16) | ((uint32_t)v[2][1] << 24);
                    const uint32_t w2 = v[2][2] | (v[3][0] << 8) | (v[3][1] << 16) | ((uint32_t)v[3][2] << 24);
                    const u32x3    q  = {w0, w1, w2};
                    __builtin_amdgcn_raw_buffer_store_b96(q, orsrc, (y * win_w + ox0) * 3, 0, 0);
                    continue;
                }
                if (KM == KM_RAW || KM == KM_STATS) { // HWC uint8, source channel order
                    const int base = (y * win_w + ox0) * cn;
#pragma unroll
                    for (int k = 0; k < 4; k++)
#pragma unroll
                        for (int c = 0; c < 3; c++)
                            if (k < nk && c < cn)
                                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)u8_of(val[k][c]), orsrc, base + k * cn + c,
                                                                     0, 0);
                    continue;
                }
                // image::loader::load: source channel c goes to output channel oc (mixChannels
                // from_to {0,2,1,1,2,0} when bgr_to_rgb); the LUT is indexed by source channel
                if (OF == OF_F32_CHW_VEC) {
                    const int idx = y * win_w + ox0;
#pragma unroll
                    for (int c = 0; c < 3; c++) {
                        const int oc = bgr ? 2 - c : c;
                        store_f32x4(orsrc, (oc * plane + idx) * 4, lut_of(c, val[0][c]), lut_of(c, val[1][c]),
                                    lut_of(c, val[2][c]), lut_of(c, val[3][c]));
                        // one channel's four LUT reads in flight at a time: hoisting all twelve
                        // costs ~20 VGPRs (two waves per SIMD) for no measurable overlap
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    continue;
                }
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    if (c >= cn) break;
                    const int oc = bgr ? 2 - c : c;
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        if (k >= nk) break;
                        const int i = a.channel_major ? oc * plane + y * win_w + ox0 + k
                                                      : (y * win_w + ox0 + k) * cn + oc;
                        if (a.out_dtype == OUT_F32)
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lut_of(c, val[k][c])), orsrc,
                                                                  i * 4, 0, kStoreAux);
                        else
                            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)u8_of(val[k][c]), orsrc, i, 0, kStoreAux);
                    }
                }
            }
        }
        if (has_next) {
            // Next band: loaded only now.  Prefetching it during this band's compute would not
            // hide its latency -- waiting for those loads also waits for this band's stores (one
            // vector-memory counter) -- and would hold ~15 VGPRs across the pixel loop.
            StageGeom Gn = G;
            const int nn = band_rows(y0 + TR, Gn);
            if (Gn.nr > a.stage_rows) {
                if (tid == 0) atomicOr(a.error, 2);
                return; // uniform: every lane sees the same band geometry
            }
            Walk     wn;
            WalkStep sn;
            Prefetch pn;
            walk_init(J, Gn, tid, pitch, L.stage, nt, wn, sn);
            stage_issue(J, srsrc, Gn, sn, wn, pn);
            build_yt(y0 + TR, nn, Gn, yt0 + (buf ^ 1) * TR);
            __syncthreads(); // single staging buffer: everyone is done reading it
            stage_finish(J, srsrc, Gn, sn, wn, pn, L.stage, pitch);
            __syncthreads();
        }
        buf ^= 1;
    }

    if (KM == KM_STATS) {
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
            for (int wv = 0; wv < (nt + 63) / 64; wv++) s += (uint32_t)red[wv * 4 + tid];
            a.partials[((size_t)J.stats_slot * a.partial_stride + chunk) * 4 + tid] = s;
        }
    }
}

// ---- host-side launch helpers (stage.cpp) ----------------------------------------------------
typedef void (*KernelFn)(LaunchArgs);

template <int KM, int RM, bool TAIL>
KernelFn pick_form(bool photo, int of)
{
    if constexpr (RM == RESIZE_AREA2X) {
        // the planner splits 2x-area records with photometric stages into a resize-only pre-pass
        // and a copy pass, so these forms are never instantiated
        if (photo) return nullptr;
        return of == OF_F32_CHW_VEC ? augment_tiles<KM, RM, false, OF_F32_CHW_VEC, false>
                                    : augment_tiles<KM, RM, false, OF_GENERIC, false>;
    } else {
        if (of == OF_F32_CHW_VEC)
            return photo ? augment_tiles<KM, RM, true, OF_F32_CHW_VEC, TAIL>
                         : augment_tiles<KM, RM, false, OF_F32_CHW_VEC, TAIL>;
        return photo ? augment_tiles<KM, RM, true, OF_GENERIC, TAIL> : augment_tiles<KM, RM, false, OF_GENERIC, TAIL>;
    }
}

template <int KM>
KernelFn pick_rm(int rm, bool tail, bool photo, int of)
{
    switch (rm) {
    case RESIZE_LINEAR:
        return tail ? pick_form<KM, RESIZE_LINEAR, true>(photo, of) : pick_form<KM, RESIZE_LINEAR, false>(photo, of);
    case RESIZE_AREA2X: return pick_form<KM, RESIZE_AREA2X, false>(photo, of);
    case RESIZE_NEAREST: return pick_form<KM, RESIZE_NEAREST, false>(photo, of);
    default: return pick_form<KM, RESIZE_COPY, false>(photo, of);
    }
}

KernelFn pick_kernel(int km, int rm, bool tail, bool photo, int of)
{
    if (km == KM_FINAL) return pick_rm<KM_FINAL>(rm, tail, photo, of);
    if (km == KM_STATS) return pick_rm<KM_STATS>(rm, tail, true, OF_GENERIC);
    return pick_rm<KM_RAW>(rm, tail, false, OF_GENERIC);
}

hipError_t launch_tiles(int km, int rm, bool tail, bool photo, const LaunchArgs& a, int n_jobs, hipStream_t stream)
{
    const int      of = (a.out_dtype == OUT_F32 && a.channel_major && a.vec_ok) ? OF_F32_CHW_VEC : OF_GENERIC;
    const KernelFn fn = pick_kernel(km, rm, tail, photo, of);
    if (!fn) return hipErrorInvalidDeviceFunction;
    dim3 grid(a.max_tiles, n_jobs), block(a.threads);
    hipLaunchKernelGGL(fn, grid, block, a.lds_bytes, stream, a);
    return hipGetLastError();
}

hipError_t set_kernel_lds_limit(int bytes)
{
    for (int km = 0; km < 3; km++)
        for (int rm = 0; rm < 4; rm++)
            for (int ph = 0; ph < 4; ph++)
                for (int of = 0; of < 2; of++) {
                    const KernelFn fn = pick_kernel(km, rm, (ph & 2) != 0, (ph & 1) != 0, of);
                    if (!fn) continue;
                    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
                    if (e != hipSuccess) return e;
                }
    return hipSuccess;
}

} // namespace aeon_hip
