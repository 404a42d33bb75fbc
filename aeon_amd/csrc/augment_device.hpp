// augment_device.hpp -- device helpers shared by the tile kernel (augment_kernels.hip) and the
// record-resident contrast kernel (record_kernels.hip): LDS addressing, job access, OpenCV resize
// coefficients and pixel arithmetic, photometric stages, staging (LDS-DMA) and wave reductions.
// Build with -ffp-contract=off (see augment_kernels.hip).
#pragma once
#include <hip/hip_ext.h>
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
typedef int16_t  i16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef int32_t  i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t  i32x2 __attribute__((ext_vector_type(2)));

// Job descriptors are read through the constant address space: uniform, scalar loads.
typedef const __attribute__((address_space(4))) AugJob cjob;
__device__ __forceinline__ cjob& job_ref(const LaunchArgs& a, int job)
{
    return ((cjob*)(uintptr_t)a.jobs)[job];
}

__device__ __forceinline__ int sat_u8(int v) { return min(max(v, 0), 255); }
__device__ __forceinline__ int sat_s16(int v) { return min(max(v, -32768), 32767); }
__device__ __forceinline__ int rnd(float v) { return (int)__builtin_rintf(v); }
// saturate_cast<uchar>(float) = sat_u8(cvRound(v)) in one instruction: v_cvt_pk_u8_f32 rounds to
// nearest even (the default mode) and clamps to [0, 255]
__device__ __forceinline__ int u8rnd(float v) { return (int)__builtin_amdgcn_cvt_pk_u8_f32(v, 0u, 0u); }
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
// Typed LDS pointer from a byte address.  All LDS traffic of the kernel goes through such
// integer-derived pointers (see lds_dma).
template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T* lds_ptr(int byte_addr)
{
    return (__attribute__((address_space(3))) T*)(size_t)(uint32_t)byte_addr;
}
__device__ __forceinline__ float    lds_ldf(int byte_addr) { return *(const lds_f32*)(size_t)(uint32_t)byte_addr; }

// The job of a tile: a copy of its AugJob in one of the workgroup's two LDS job slots, brought in
// by one LDS-DMA a tile ahead (from the device job table, or straight from the caller's pinned
// slot over PCIe for single-pass calls: no planner or upload launch), its fields read as uniform
// values (ds_read + readfirstlane).  Measured equal to constant-address scalar loads of a device
// table (C2 39.9-40.6 vs 40.1-40.4 us), and it is what lets the job table live in host memory.
struct JobRef {
    int lds; // byte address of the LDS copy
};
template <typename T>
__device__ __forceinline__ T job_get(const JobRef& J, int off)
{
    if constexpr (sizeof(T) == 8) {
        const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane(lds_ld(J.lds + off));
        const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(lds_ld(J.lds + off + 4));
        return __builtin_bit_cast(T, lo | (hi << 32));
    } else {
        return __builtin_bit_cast(T, (uint32_t)__builtin_amdgcn_readfirstlane(lds_ld(J.lds + off)));
    }
}
// The hot half of a job (kJobHotBytes: every field a non-photometric tile reads) loaded from its LDS
// copy at once -- eight 16-byte LDS reads, one wait -- into scalar registers: JF on it is a register
// read, where JF on a JobRef is an LDS round trip per field (each one waited for before the next; in
// augment_split's per-tile staging those waits were most of its 1.8 us).
struct JobS {
    uint32_t w[kJobHotBytes / 4];
};
__device__ __forceinline__ JobS job_load(int lds)
{
    u32x4 v[kJobHotBytes / 16];
#pragma unroll
    for (int i = 0; i < kJobHotBytes / 16; i++) v[i] = *lds_ptr<const u32x4>(lds + 16 * i);
    JobS J;
#pragma unroll
    for (int i = 0; i < kJobHotBytes / 16; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) J.w[4 * i + k] = __builtin_amdgcn_readfirstlane(v[i][k]);
    return J;
}
template <typename T>
__device__ __forceinline__ T job_get(const JobS& J, int off)
{
    if constexpr (sizeof(T) == 8) {
        return __builtin_bit_cast(T, (uint64_t)J.w[off >> 2] | ((uint64_t)J.w[(off >> 2) + 1] << 32));
    } else {
        return __builtin_bit_cast(T, J.w[off >> 2]);
    }
}
#define JF(J, field) job_get<decltype(AugJob::field)>(J, (int)__builtin_offsetof(AugJob, field))
#define JFA(J, field, i)                                                                                     \
    job_get<__remove_extent(decltype(AugJob::field))>(J, (int)__builtin_offsetof(AugJob, field) +           \
                                                             (int)sizeof(AugJob::field[0]) * (i))

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

// 24-bit signed multiply-add, full rate.  Spelled in asm: for __mul24 the backend sometimes
// sign-extends on the scalar unit and then selects the quarter-rate v_mul_lo_u32.  Callers
// guarantee |operands| < 2^23.
__device__ __forceinline__ int mad_i24(int a, int b, int c)
{
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ---- photometric stages (aeon src/image.cpp:336-406 over OpenCV 2.4) ------------------------
// The cv::transform coefficients of the tile's record, copied once per tile into VGPRs (the
// fixed-point ones for BS_FIXPT, the float ones' bits otherwise): held in SGPRs the compiler
// re-loads them per pixel under SGPR pressure, and every such scalar load's lgkmcnt(0) wait
// also drains the pixel's LDS reads.
struct BsRegs {
    uint32_t w[9];
};
__device__ __forceinline__ uint32_t to_vgpr(uint32_t s)
{
    uint32_t v;
    asm("v_mov_b32 %0, %1" : "=v"(v) : "s"(s));
    return v;
}
// BS_FIXPT keeps the coefficients of B and G as int16 pairs, (q0, q1), (q3, q4), (q6, q7), for
// v_dot2_i32_i16, and the R ones (q2, q5, q8) as plain words.
__device__ __forceinline__ BsRegs bs_regs(const JobRef& J)
{
    BsRegs R;
    if (JF(J, bs_kind) == BS_FIXPT) {
#pragma unroll
        for (int i = 0; i < 3; i++) {
            R.w[i]     = to_vgpr(((uint32_t)JFA(J, bsq, 3 * i) & 0xffffu) | ((uint32_t)JFA(J, bsq, 3 * i + 1) << 16));
            R.w[3 + i] = to_vgpr((uint32_t)JFA(J, bsq, 3 * i + 2));
        }
        R.w[6] = R.w[7] = R.w[8] = 0;
    } else {
#pragma unroll
        for (int k = 0; k < 9; k++) R.w[k] = to_vgpr(__float_as_uint(JFA(J, bsm, k)));
    }
    return R;
}
__device__ __forceinline__ void bs_apply(int kind, const BsRegs& R, int& b, int& g, int& r)
{
    const auto m = [&](int k) { return __uint_as_float(R.w[k]); };
    if (kind == BS_DIAG) { // diagtransform_8u
        b = u8rnd(m(0) * (float)b + 0.f);
        g = u8rnd(m(4) * (float)g + 0.f);
        r = u8rnd(m(8) * (float)r + 0.f);
    } else if (kind == BS_FIXPT) { // transform_8u, 10-bit fixed point
        // |q| < 2^15, x < 2^8: exact in int32 in any order.  q_B*b + q_G*g as one v_dot2_i32_i16
        // on the (b, g) pair, + q_R*r + 512 as a full-rate 24-bit multiply-add.
        const i16x2 bg = __builtin_bit_cast(i16x2, (uint32_t)b | ((uint32_t)g << 16));
        const auto  dq = [&](int i, int acc) { return __builtin_amdgcn_sdot2(bg, __builtin_bit_cast(i16x2, R.w[i]), acc, false); };
        int t0 = dq(0, mad_i24((int)R.w[3], r, 512)) >> 10;
        int t1 = dq(1, mad_i24((int)R.w[4], r, 512)) >> 10;
        int t2 = dq(2, mad_i24((int)R.w[5], r, 512)) >> 10;
        b = sat_u8(t0), g = sat_u8(t1), r = sat_u8(t2);
    } else { // transform_<uchar,float>
        float fb = (float)b, fg = (float)g, fr = (float)r;
        b = u8rnd(m(0) * fb + m(1) * fg + m(2) * fr + 0.f);
        g = u8rnd(m(3) * fb + m(4) * fg + m(5) * fr + 0.f);
        r = u8rnd(m(6) * fb + m(7) * fg + m(8) * fr + 0.f);
    }
}


// cvtColor(BGR2HSV) [RGB2HSV_b], H = (H + hue) % 180 stored as uchar, cvtColor(HSV2BGR)
// [HSV2RGB_b over HSV2RGB_f].  HSV2RGB_f's sector and fraction depend only on the uchar H, and
// each output channel is one of t0 = v, t1 = v(1-s), t2 = v(1-s*f), t3 = v(1-s(1-f)), i.e.
// v*(1 - s*w) with w in {0, 1, f, 1-f}: a 256-entry table of per-channel weights (B, G, R, 0),
// built on the host with HSV2RGB_f's own float operations, gives every t exactly (s*0 = 0,
// s*1 = s, and 1-f rounded once as OpenCV does).  With s == 0 every t equals v exactly, so
// OpenCV's s == 0 branch needs no special case.
#ifndef AEON_HIP_HUE_BATCH
#define AEON_HIP_HUE_BATCH 2
#endif
constexpr int kHueBatch = AEON_HIP_HUE_BATCH; // pixels per hue_apply_n (1, 2 or 4)
// Over N of a lane's 4 pixels at once: the 2N division-table reads (sdiv[v], hdiv[diff]) and
// then the N weight-table reads are issued back to back, so one LDS latency is waited for per
// group of reads instead of one per read (the per-pixel form waited three times per pixel).
// htab = the tile's hue table at h12 = 0 (kHueTabBytes): OpenCV's h (h12 below, in [-30, 150] for
// every BGR triple, tools/hue_range.py) -> its +180 wrap, + hue, % 180 stored as uchar, -> the
// HSV2RGB weights of that H, all folded into the one lookup.
template <int N, int K0, typename STAB, typename TAB, typename WTAB>
__device__ __forceinline__ void hue_apply_n(STAB sdv, TAB hdiv, WTAB htab, int (&pxs)[4][3])
{
    int (*px)[3] = pxs + K0; // pixels K0 .. K0 + N - 1
    int v[N], diff[N], sd[N], hd[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        const int b = px[k][0], g = px[k][1], r = px[k][2];
        v[k]        = max(b, max(g, r));
        diff[k]     = v[k] - min(b, min(g, r));
    }
#pragma unroll
    for (int k = 0; k < N; k++) sd[k] = sdv[v[k]].x, hd[k] = hdiv[diff[k]];
    int   h12[N];
    float sf[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        const int b = px[k][0], g = px[k][1], r = px[k][2];
        const int vr = v[k] == r ? -1 : 0, vg = v[k] == g ? -1 : 0;
        // operands < 2^23 in magnitude (sdiv <= 255<<12, hdiv <= 30<<12, |h| <= 5*255)
        const int s = mad_i24(diff[k], sd[k], 1 << 11) >> 12;
        int h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff[k])) + ((~vg) & (r - g + 4 * diff[k]))));
        h12[k] = mad_i24(h, hd[k], 1 << 11) >> 12;
        sf[k] = (float)s * (1.f / 255);
    }
    f32x4 w[N];
#pragma unroll
    for (int k = 0; k < N; k++) w[k] = htab[h12[k]];
#pragma unroll
    for (int k = 0; k < N; k++) {
        const float vf = (float)v[k] * (1.f / 255);
#if defined(AEON_HIP_EXP_HUE_NOTAIL) // development ablation: no HSV2RGB float chain (wrong values)
        px[k][0] = (int)w[k][0] + v[k], px[k][1] = (int)w[k][1] + (int)sf[k], px[k][2] = (int)w[k][2];
#else
        // v, s in [0, 1] and w in [0, 1]: every product is in [0, 255], no saturation needed
        px[k][0] = u8rnd(vf * (1.f - sf[k] * w[k][0]) * 255.f);
        px[k][1] = u8rnd(vf * (1.f - sf[k] * w[k][1]) * 255.f);
        px[k][2] = u8rnd(vf * (1.f - sf[k] * w[k][2]) * 255.f);
#endif
    }
}

// The division tables in LDS (kHsvLdsDivBytes): {sdiv[v], (float)v * (1.f / 255)} pairs, hdiv180.
__device__ __forceinline__ void hsv_div_tables(const LdsLayout& L, const int32_t* g)
{
    const auto sdv = lds_ptr<i32x2>(L.hsv);
    const auto hd  = lds_ptr<int32_t>(L.hsv + 256 * 8);
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        sdv[i] = (i32x2){g[i], (int)__float_as_uint((float)i * (1.f / 255))};
        hd[i]  = g[256 + i];
    }
}

// hue_apply_n for the SPEC_BS_HUE pass-1 loop, the result packed as one dword (B, G, R, 0) per
// pixel.  In every HSV2RGB_f sector one output channel is t0 = v (w = 0: v/255*255 rounds back to
// v for all 256 v), one is t1 = v(1-s) (w = 1, s*1 == s) and one is v(1 - s*w) with w in {f, 1-f}:
// the tile's table entry (htab8 at h12) = {bits of that w, v_perm selector placing (v, t1, t_w)
// in the channel order}; the two float chains are OpenCV's own operations, so every byte equals
// hue_apply_n's.
template <int N, int K0, typename STAB, typename TAB, typename ETAB>
__device__ __forceinline__ void hue_pack_n(STAB sdv, TAB hdiv, ETAB htab8, const int (&pxs)[4][3], uint32_t (&pk)[4])
{
    const int (*px)[3] = pxs + K0;
    int   v[N], diff[N], hd[N];
    i32x2 sv[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        const int b = px[k][0], g = px[k][1], r = px[k][2];
        v[k]        = max(b, max(g, r));
        diff[k]     = v[k] - min(b, min(g, r));
    }
#pragma unroll
    for (int k = 0; k < N; k++) sv[k] = sdv[v[k]], hd[k] = hdiv[diff[k]];
    int   h12[N];
    float sf[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        const int b = px[k][0], g = px[k][1], r = px[k][2];
        const int vr = v[k] == r ? -1 : 0, vg = v[k] == g ? -1 : 0;
        const int s = mad_i24(diff[k], sv[k].x, 1 << 11) >> 12;
        int h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff[k])) + ((~vg) & (r - g + 4 * diff[k]))));
        h12[k] = mad_i24(h, hd[k], 1 << 11) >> 12;
        sf[k]  = (float)s * (1.f / 255);
    }
    i32x2 e[N];
#pragma unroll
    for (int k = 0; k < N; k++) e[k] = htab8[h12[k]];
#pragma unroll
    for (int k = 0; k < N; k++) {
        const float vf = __uint_as_float((uint32_t)sv[k].y);
#ifndef AEON_HIP_HUE_PK_F32
#define AEON_HIP_HUE_PK_F32 1
#endif
#if AEON_HIP_HUE_PK_F32 // both chains as packed f32 (s*1 == s exactly; separate IEEE mul/add, no FMA)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        f32x2       t  = (f32x2){sf[k], sf[k]} * (f32x2){1.f, __uint_as_float((uint32_t)e[k].x)};
        t              = ((1.f - t) * vf) * 255.f;
        const float c1 = t.x, cw = t.y;
#else
        const float c1 = vf * (1.f - sf[k]) * 255.f;
        const float cw = vf * (1.f - sf[k] * __uint_as_float((uint32_t)e[k].x)) * 255.f;
#endif
        uint32_t    q  = __builtin_amdgcn_cvt_pk_u8_f32(c1, 1u, (uint32_t)v[k]);
        q              = __builtin_amdgcn_cvt_pk_u8_f32(cw, 2u, q);
        pk[K0 + k]     = __builtin_amdgcn_perm(0u, q, (uint32_t)e[k].y);
    }
}

// Sum over the 64 lanes of a full wave with DPP adds (no LDS permutes), uniform result: quad
// permutes and row mirrors give every lane its row's sum, row_bcast:15 / :31 carry rows 0..2
// into rows 1..3, lane 63 holds the total.  Integer adds: exact in any order.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    v += dpp_u32<0xb1>(v);       // quad_perm [1, 0, 3, 2]
    v += dpp_u32<0x4e>(v);       // quad_perm [2, 3, 0, 1]
    v += dpp_u32<0x141>(v);      // row_half_mirror
    v += dpp_u32<0x140>(v);      // row_mirror
    v += dpp_u32<0x142, 0xa>(v); // row_bcast:15 -> rows 1, 3
    v += dpp_u32<0x143, 0xc>(v); // row_bcast:31 -> rows 2, 3
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// ---- source staging (LDS-DMA) ------------------------------------------------------------------
// A tile (a band of TR output rows of one record) needs source rows [v_lo, v_lo+nr) x cols
// [u_lo, u_lo+nc), staged as one 32-bit word per pixel (B, G, R, x), rows `pitch` = 4*ng words
// apart (ng = ceil(nc/4) groups of 4 pixels), in one of the workgroup's two LDS staging buffers.
// (1) LDS-DMA, no VGPR round trip: for BGR, group q = j*ng + g is loaded by lane q%64 of
// wave-instruction q/64 as the 12 bytes at its exact, unaligned source offset; a dwordx3 LDS-DMA
// lands each lane's 12 bytes in a 16-byte slot (measured, tools/probes/glds_probe.py), i.e. exactly
// where the group's four words go.  For one channel: one pixel per lane, 4 bytes from its own
// offset (bytes 1-3 ignored).  The next tile's loads are issued before the current tile is
// computed.  (2) After the issuing wave's own vmcnt wait, each lane unpacks the BGR slots it
// loaded, in place.  The byte-exact rules are applied in (2): pixels outside the crop of a padded
// job are 0 (add_padding's border); a load that crossed the end of the source buffer (a buffer
// load past num_records returns 0 for the whole access) is re-read byte by byte.
constexpr uint32_t kOutOfRange = 0x80000000u;

// buffer_load_dwordx3 ... lds: lane l -> LDS bytes lds_base + 16*l (12 written);
// buffer_load_dword ... lds: lane l -> lds_base + 4*l.  Inline asm on purpose: hipcc tracks its
// own LDS-DMA builtins and then waits vmcnt(0) before LDS reads inside the compute loops (they
// may alias, as far as it can tell), which would drain the next tile's loads at the first pixel.
// The kernel orders these loads itself: counted vmcnt, then a barrier.  M0 is set here and used
// by nothing else in these kernels.
template <int BYTES>
__device__ __forceinline__ void lds_dma(__amdgpu_buffer_rsrc_t rsrc, int lds_base, uint32_t voff)
{
    if (BYTES == 12)
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx3 %1, %2, 0 offen lds"
                     :
                     : "s"(__builtin_amdgcn_readfirstlane(lds_base)), "v"(voff), "s"(rsrc)
                     : "memory");
    else
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds"
                     :
                     : "s"(__builtin_amdgcn_readfirstlane(lds_base)), "v"(voff), "s"(rsrc)
                     : "memory");
}

// Buffer resource with its fields forced into scalar registers (the LDS-DMA asm takes an SGPR
// quad; the values are uniform, but the compiler cannot always prove it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int bytes)
{
    const uint64_t v  = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0,
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

struct StageGeom { // uniform: the staged source of one tile
    int v_lo, nr, u_lo, nc, ng, pitch; // rows [v_lo, v_lo + nr), columns [u_lo, u_lo + nc), pitch = 4 * ng
    int rp;                            // LDS bytes per staged row
};

// The LDS image of a tile's staged rows (stage_bytes_for, aug_job.hpp): the rows' units (BGR groups
// of 4 pixels as 16-byte slots, or gray pixels as words) back to back, rp = 16 * ng bytes per row,
// loaded by whole 64-unit DMA instructions.  (Row-aligned instructions -- every row in its own whole
// instructions, so a lane's source offset is a row base + lane * unit bytes -- measured slower: a
// 256-wide crop needs 65 groups per row, i.e. two instructions, and the doubled LDS cuts C2's
// rows per tile from 32 to 19: 46.3 vs 40.1 us.)
__device__ __forceinline__ void stage_layout(int cn, StageGeom& G) { G.rp = G.pitch * 4; }
__device__ __forceinline__ int stage_need(const StageGeom& G, int cn)
{
    return cn == 3 ? (G.nr * G.ng + 63) / 64 * 1024 : (G.nr * G.pitch + 63) / 64 * 256;
}

// byte offset in the source buffer of staged pixel (row j, column u); negative above/left of a
// padded crop
template <typename JR>
__device__ __forceinline__ int src_off(const JR& J, const StageGeom& G, int j, int u)
{
    return (JF(J, crop_y) + G.v_lo + JF(J, shift_y) + j) * JF(J, src_stride) + (JF(J, crop_x) + G.u_lo + JF(J, shift_x) + u) * JF(J, cn);
}

// Units (BGR groups or gray pixels) per staged row.
template <typename JR>
__device__ __forceinline__ int stage_units_per_row(const JR& J, const StageGeom& G) { return JF(J, cn) == 3 ? G.ng : G.pitch; }

// (1) This wave's share of the tile's LDS-DMA loads: instructions wave, wave + nw, ...; unit q of
// the tile (row q / upr) lands in slot q.
template <typename JR>
__device__ __forceinline__ void stage_issue(const JR& J, const StageGeom& G, int buf, int wave, int nw)
{
    const int   lane = threadIdx.x & 63;
    const int   cn   = JF(J, cn);
    const auto  rsrc = uniform_rsrc((const void*)JF(J, src_ptr), (int)JF(J, src_bytes));
    const int   upr  = stage_units_per_row(J, G);
    const int   Q    = G.nr * upr;
    const int   ub   = cn == 3 ? 12 : 1; // source bytes per unit
    const int   row0 = src_off(J, G, 0, 0);
    const int   rs   = JF(J, src_stride);
    const float inv  = 1.f / (float)upr;
    for (int i = wave; i * 64 < Q; i += nw) {
        const int q    = i * 64 + lane;
        uint32_t  voff = kOutOfRange;
        if (q < Q) {
            const int j = (int)(((float)q + 0.5f) * inv); // exact in f32 for q < 2^20
            const int b = row0 + j * rs + (q - j * upr) * ub;
            voff        = b >= 0 ? (uint32_t)b : kOutOfRange; // (padded jobs: fixed in stage_unpack)
        }
        if (cn == 3) lds_dma<12>(rsrc, buf + i * 1024, voff);
        else lds_dma<4>(rsrc, buf + i * 256, voff);
    }
}

// (2) After this wave's loads landed: unpack its BGR slots in place; zero border of a padded job;
// re-read loads that crossed the end of the buffer (rare; uniformly skipped otherwise for gray).
__device__ __forceinline__ u32x4 unpack_bgr(u32x4 w) // 12 bytes BGR BGR BGR BGR -> four (B, G, R, 0) words
{
    return (u32x4){w.x & 0xffffffu, __builtin_amdgcn_perm(w.y, w.x, 0x0C050403u),
                   __builtin_amdgcn_perm(w.z, w.y, 0x0C040302u), w.z >> 8};
}
template <typename JR>
__device__ __forceinline__ void stage_unpack(const JR& J, const StageGeom& G, int buf, int wave, int nw)
{
    const int  lane      = threadIdx.x & 63;
    const int  cn        = JF(J, cn);
    const int  src_bytes = (int)JF(J, src_bytes);
    const bool padded    = JF(J, padded) != 0;
    const bool at_end    = src_off(J, G, G.nr - 1, G.pitch) + 12 > src_bytes;
    if (cn != 3 && !padded && !at_end) return;
    const int   upr = stage_units_per_row(J, G);
    const int   Q   = G.nr * upr;
    if (cn == 3 && !padded && !at_end) {
        // common case: in-place unpack of this wave's slots, reads of several instructions in
        // flight before their writes
        int i = wave;
        for (; (i + 2 * nw) * 64 < Q; i += 3 * nw) {
            u32x4 w[3];
#pragma unroll
            for (int k = 0; k < 3; k++) w[k] = *lds_ptr<const u32x4>(buf + ((i + k * nw) * 64 + lane) * 16);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                const int q = (i + k * nw) * 64 + lane;
                if (q < Q) *lds_ptr<u32x4>(buf + q * 16) = unpack_bgr(w[k]);
            }
        }
        for (; i * 64 < Q; i += nw) {
            const int q = i * 64 + lane;
            if (q >= Q) continue;
            const auto slot = lds_ptr<u32x4>(buf + q * 16);
            *slot           = unpack_bgr(*slot);
        }
        return;
    }
    const float inv = 1.f / (float)upr;
    for (int i = wave; i * 64 < Q; i += nw) {
        const int q = i * 64 + lane;
        if (q >= Q) continue;
        const int j  = (int)(((float)q + 0.5f) * inv);
        const int u0 = (q - j * upr) * (cn == 3 ? 4 : 1); // first staged column of this unit
        const int np = cn == 3 ? 4 : 1;                   // pixels of this unit
        const int b  = src_off(J, G, j, u0);
        const bool slow = padded || b < 0 || (at_end && b + (cn == 3 ? 12 : 4) > src_bytes);
        if (cn == 3 && !slow) {
            const auto slot = lds_ptr<u32x4>(buf + q * 16);
            *slot           = unpack_bgr(*slot);
        } else if (slow) {
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)JF(J, src_ptr), (short)0, src_bytes, 0x00020000);
            for (int k = 0; k < np; k++) {
                const int cy = G.v_lo + j + JF(J, shift_y), cx = G.u_lo + u0 + k + JF(J, shift_x);
                uint32_t  p  = 0;
                if (!padded || (cy >= 0 && cy < JF(J, crop_h) && cx >= 0 && cx < JF(J, crop_w))) {
                    const int bb = b + k * cn;
                    if (bb >= 0)
                        for (int c = 0; c < cn; c++)
                            p |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, bb + c, 0, 0) << (8 * c);
                }
                *lds_ptr<uint32_t>(buf + (q * np + k) * 4) = p;
            }
        }
    }
}

// The job descriptor of tile t into an LDS job slot: one 64-lane LDS-DMA of its a.job_bytes (256, or
// the 128 hot bytes when no job of the launch has photometric stages).  A job table in pinned host
// memory (a.jobs_host) is read through to the host (sc0 sc1: the host wrote the slot since the GPU
// last read it).
__device__ __forceinline__ void fetch_job(const LaunchArgs& a, int t, int lds_slot)
{
    if (t < 0 || t >= a.total_tiles) return;
    const int      job  = t / a.max_tiles;
    const auto     rs   = uniform_rsrc((const void*)((const char*)a.jobs + (size_t)job * a.job_stride), a.job_bytes);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t voff = lane * 4 < (uint32_t)a.job_bytes ? lane * 4 : kOutOfRange; // (the rest of the slot: 0)
    const int      base = __builtin_amdgcn_readfirstlane(lds_slot);
    if (a.jobs_host)
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen sc0 sc1 lds" : : "s"(base), "v"(voff), "s"(rs)
                     : "memory");
    else
        lds_dma<4>(rs, lds_slot, voff);
}

// Wait until at most n vector-memory instructions of this wave are outstanding (the immediate
// must be a constant: buckets, rounding n down).
__device__ __forceinline__ void wait_vm_upto(int n)
{
    if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Workgroup barrier that leaves vector-memory operations in flight (__syncthreads() would drain
// vmcnt): LDS writes are made visible (lgkmcnt 0) and the compiler may not move memory
// operations across it.
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// Output cache policy: streaming stores (written once, read by the consumer of the batch).
#ifndef AEON_HIP_STORE_AUX
#define AEON_HIP_STORE_AUX 2 // nt
#endif
constexpr int kStoreAux = AEON_HIP_STORE_AUX;
#ifndef AEON_HIP_STAGE_PRIO
#define AEON_HIP_STAGE_PRIO 1
#endif
#ifndef AEON_HIP_COMPUTE_PRIO
#define AEON_HIP_COMPUTE_PRIO 0
#endif
constexpr int kStagePrio   = AEON_HIP_STAGE_PRIO;   // s_setprio of a tile's staging phases
constexpr int kComputePrio = AEON_HIP_COMPUTE_PRIO; // ... and of its compute/store phase

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
__device__ __forceinline__ void resize_px(i32x4 ytr, int col, uint32_t wx, int s[3])
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

// resize_px<RESIZE_LINEAR, true> for a lane's 4 pixels of a row with all 16 staged words read first: the
// reads are in flight together (one LDS wait per row instead of one per pixel).
template <bool SCALED = true>
__device__ __forceinline__ void resize4_linear(i32x4 ytr, const int (&col)[4], const uint32_t (&wx)[4], int (&s)[4][3])
{
    uint32_t p[4][4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int a0 = ytr.x + col[q], a1 = ytr.y + col[q];
        p[q][0] = lds_ld(a0), p[q][1] = lds_ld(a0 + 4), p[q][2] = lds_ld(a1), p[q][3] = lds_ld(a1 + 4);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const u16x2 w = __builtin_bit_cast(u16x2, wx[q]);
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const uint32_t sel = (uint32_t)c | (0x0Cu << 8) | ((4u + c) << 16) | (0x0Cu << 24);
            const uint32_t H0  = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p[q][1], p[q][0], sel)), w, 0u, false);
            const uint32_t H1  = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(p[q][3], p[q][2], sel)), w, 0u, false);
            const uint32_t t0  = (uint32_t)__mul24((int)(H0 >> 4), ytr.z) + (2u << 16);
            const uint32_t t1  = (uint32_t)__mul24((int)(H1 >> 4), ytr.w);
            s[q][c]            = (int)((t0 >> 16) + (t1 >> 16));
            if (!SCALED) s[q][c] >>= 2;
        }
    }
}
__device__ __forceinline__ void resize4_linear_scaled(i32x4 ytr, const int (&col)[4], const uint32_t (&wx)[4], int (&s)[4][3])
{
    resize4_linear<true>(ytr, col, wx, s);
}

// Elements of OpenCV's scalar row tail (e >= xv) use FixedPtCast<int, uchar, 22> instead.
template <bool SCALED>
__device__ __forceinline__ void tail_fix(i32x4 ytr, int col, uint32_t wx, int e0, int xv, int s[3])
{
    const uint32_t p00 = lds_ld(ytr.x + col), p01 = lds_ld(ytr.x + col + 4);
    const uint32_t p10 = lds_ld(ytr.y + col), p11 = lds_ld(ytr.y + col + 4);
    const int      a0 = wx & 0xffff, a1 = (int)(wx >> 16);
    for (int c = 0; c < 3; c++) {
        if (e0 + c < xv) continue;
        const int H0 = __mul24(byte_of(p00, c), a0) + __mul24(byte_of(p01, c), a1);
        const int H1 = __mul24(byte_of(p10, c), a0) + __mul24(byte_of(p11, c), a1);
        s[c]         = sat_u8((__mul24(H0, ytr.z) + __mul24(H1, ytr.w) + (1 << 21)) >> 22) << (SCALED ? 2 : 0);
    }
}

// standardize LUT (LDS offset 0) entry for source channel c at scaled value s
#ifdef AEON_HIP_EXP_NOLUT // development ablation: no LUT reads (wrong values)
__device__ __forceinline__ float lut_at(int c, int s) { return (float)(s + c); }
#else
__device__ __forceinline__ float lut_at(int c, int s) { return lds_ldf(c * 1024 + (s & ~3)); }
#endif

} // namespace aeon_hip
