// record_kernels.hip -- contrast records in ONE launch, the post-hue record held in registers.
//
// photometric::cbsjitter's contrast (aeon src/image.cpp:398-405) needs the mean of the post-hue
// image before any output value: the two-launch path writes that image to HBM (pass 1, KM_STATS)
// and reads it back (pass 2), 2 x 150 KB per 224x224 record on top of the record's own bytes.  Here a
// persistent workgroup per CU takes whole records, and a record's post-hue pixels never leave the
// chip: each of the workgroup's lanes owns 4 output columns of one row in every 16 (row phase) and
// keeps its 12 bytes per row -- up to 14 rows, 42 VGPRs -- in registers.  The workgroup's records
// form a pipeline of steps; step k interleaves, tile by tile (32 output rows, two per lane),
//   A(k):   record k's resize -> brightness/saturation -> hue (the contrast pass-1 arithmetic of
//           augment_tiles, from LDS-DMA-staged source rows, double-buffered) into the lane's
//           registers, plus its exact channel sums, and
//   B(k-1): record k-1's output rows from the registers through its per-record table (contrast ->
//           lighting -> standardize, built once the sums of the whole record are known), stored as
//           float4 planes, so that B's store stream drains while A computes (VALU-bound) -- the two
//           kinds of work of the two-launch path overlap inside every CU.
// After step k's tiles the sums give (1-c)*mean in f64 (contrast_reduce's arithmetic) and record k's
// table.  The registers rotate by one tile per tile (B reads the oldest tile's 6 dwords, A appends
// the newest), so all register indices are compile-time constants.
// Every byte equals the two-launch path's (tests: test_full_batch_c3_all_records and the C3 cases).
#include "augment_device.hpp"

// development ablations / variants (tools/build_variants.sh): HUE4 = four pixels per hue batch;
// NOB / NOA = no B stores / no A compute (wrong outputs)
#ifndef AEON_REC_HUE4
#define AEON_REC_HUE4 0
#endif
#ifndef AEON_REC_NOB
#define AEON_REC_NOB 0
#endif
#ifndef AEON_REC_NOA
#define AEON_REC_NOA 0
#endif
#ifndef AEON_REC_HELPER_PRIO // s_setprio of the split kernel's helper waves
#define AEON_REC_HELPER_PRIO 3
#endif
#ifndef AEON_REC_UNROLL // split kernel: the compute waves' tile loop unrolled (no register rotation)
#define AEON_REC_UNROLL 1
#endif
#ifndef AEON_REC_HOIST // FAST form: a row's 16 tap words read together (resize4_linear)
#define AEON_REC_HOIST 1
#endif
#ifndef AEON_REC_FUSED // FAST form: A and B of a row interleaved (rec_row_fast); 0 = B's row, then A's
#define AEON_REC_FUSED 1
#endif

namespace aeon_hip {

namespace {

// The job of record `job` into LDS slot `slot` by one wave's LDS-DMA (wave 0; from the pinned slot
// over PCIe with sc0 sc1 when a.jobs_host, as fetch_job).
__device__ __forceinline__ void rec_fetch_job(const LaunchArgs& a, int job, int slot)
{
    const auto     rs   = uniform_rsrc((const void*)(a.jobs + job), (int)sizeof(AugJob));
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t voff = lane * 4;
    const int      base = __builtin_amdgcn_readfirstlane(slot);
    if (a.jobs_host)
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen sc0 sc1 lds" : : "s"(base), "v"(voff), "s"(rs)
                     : "memory");
    else
        lds_dma<4>(rs, slot, voff);
}

struct RecTile {
    bool      ok;
    int       y0, nrows;
    StageGeom G;
};

// staged-source geometry of tile `band` (rows band*32 ...) of the record whose job is J
template <typename JR>
__device__ __forceinline__ RecTile rec_tile(const JR& J, int band, int TR, int H, int stage_bytes, int32_t* error)
{
    RecTile f;
    f.ok    = false;
    f.y0    = band * TR;
    f.nrows = min(TR, H - f.y0);
    if (f.nrows <= 0) return f;
    const XTap xf = xcoef<RESIZE_LINEAR>(JF(J, win_x), JF(J, scale_x), JF(J, crop_w));
    const XTap xl = xcoef<RESIZE_LINEAR>(JF(J, win_x) + JF(J, win_w) - 1, JF(J, scale_x), JF(J, crop_w));
    StageGeom& G  = f.G;
    G.u_lo  = xf.sx;
    G.nc    = xl.sx + 1 - G.u_lo + 1;
    G.ng    = (G.nc + 3) >> 2;
    G.pitch = 4 * G.ng;
    G.v_lo  = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0, JF(J, scale_y), JF(J, crop_h)).r0;
    G.nr    = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0 + f.nrows - 1, JF(J, scale_y), JF(J, crop_h)).r1 - G.v_lo + 1;
    stage_layout(3, G);
    if (stage_need(G, 3) > stage_bytes) {
        if (error && (threadIdx.x & 63) == 0) atomicOr(error, 2);
        return f;
    }
    f.ok = true;
    return f;
}

// row taps of tile f into the table at yt (staged rows in the buffer at `stage`)
template <typename JR>
__device__ __forceinline__ void rec_row_taps(const JR& J, const RecTile& f, int yt, int stage, int i0, int step)
{
    for (int r = i0; r < f.nrows; r += step) {
        const YTap y = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0 + r, JF(J, scale_y), JF(J, crop_h));
        lds_ptr<i32x4>(yt)[r] = (i32x4){stage + (y.r0 - f.G.v_lo) * f.G.rp, stage + (y.r1 - f.G.v_lo) * f.G.rp, y.b0, y.b1};
    }
}

// The A record's column taps (flip folded in: the lane's output column ox reads source column x)
// and hue table (Bands::tables' two forms), by the whole workgroup.
__device__ __forceinline__ void rec_record_tables(const LaunchArgs& a, const RecLds& L, const JobRef& J, int W, bool fast)
{
    const int tid = threadIdx.x, nt = blockDim.x;
    const auto xt = lds_ptr<i32x2>(L.xt);
    int        u_lo = xcoef<RESIZE_LINEAR>(JF(J, win_x), JF(J, scale_x), JF(J, crop_w)).sx;
    for (int x = tid; x < W; x += nt) {
        const XTap c = xcoef<RESIZE_LINEAR>(JF(J, win_x) + x, JF(J, scale_x), JF(J, crop_w));
        xt[x]        = (i32x2){4 * (c.sx - u_lo), (c.a0 & 0xffff) | (c.a1 << 16)};
    }
    if (!(JF(J, photo) & PHOTO_HUE)) return;
    const auto   wt  = lds_ptr<const f32x4>(L.hwt);
    const int    hue = JF(J, hue);
    const bool   sp  = fast;
    for (int i = tid; i < kHueTabEntries; i += nt) {
        const int   h12 = i - 30;
        const f32x4 w   = wt[(((h12 < 0 ? h12 + 180 : h12) + hue) % 180) & 0xff];
        if (!sp) {
            lds_ptr<f32x4>(L.htab)[i] = w;
            continue;
        }
        const int iv = w[0] == 0.f ? 0 : (w[1] == 0.f ? 1 : 2);
        int       i1 = -1;
        for (int c = 0; c < 3; c++)
            if (c != iv && i1 < 0 && w[c] == 1.f) i1 = c;
        if (i1 < 0) i1 = iv == 0 ? 1 : 0, atomicOr(a.error, 16);
        const int iw  = 3 - iv - i1;
        uint32_t  sel = 0x0c000000u;
        for (int c = 0; c < 3; c++) sel |= (uint32_t)(c == iv ? 0 : (c == i1 ? 1 : 2)) << (8 * c);
        lds_ptr<i32x2>(L.htab)[i] = (i32x2){(int)__float_as_uint(w[iw]), (int)sel};
    }
}

// Record k's table: y -> contrast (with its (1-c)*mean from the exact sums) -> lighting ->
// standardize (the LUT in global memory), Bands::record_table's arithmetic.
__device__ __forceinline__ void rec_table(const LaunchArgs& a, const RecLds& L, const JobRef& J, int W, int H, int nw,
                                          int sums_at)
{
    const int photo = JF(J, photo);
    const auto ps   = lds_ptr<const uint32_t>(sums_at);
    uint32_t   s[3] = {0, 0, 0};
    for (int w = 0; w < nw; w++)
        for (int c = 0; c < 3; c++) s[c] += ps[w * 4 + c];
    // contrast_reduce: cv::mean = sum * (1./N) in f64, times (1 - c)
    // (N from the job's LDS copy, not the kernel's W*H: a loop-invariant double would be hoisted out of
    // the record loop and spilled, and its scratch reload waits for every store in flight)
    const double inv_n = 1. / (double)(JF(J, win_w) * JF(J, win_h));
    const double kc    = 1.0 - (double)JF(J, contrast);
    double       sh[3];
    for (int c = 0; c < 3; c++) sh[c] = kc * ((double)s[c] * inv_n);
    const float c = JF(J, contrast), la = JF(J, light_a);
    const auto  rt = lds_ptr<float>(L.rtab);
    for (int i = threadIdx.x; i < 3 * 256; i += blockDim.x) {
        const int ch = i >> 8;
        int       y  = i & 255;
        if (photo & PHOTO_CONTRAST) y = u8rnd((float)((double)((float)y * c + 0.f) + sh[ch]));
        if (photo & PHOTO_LIGHTING) y = sat_u8(u8rnd((float)y * la + 0.f) + JFA(J, light_add, ch));
        rt[i] = lds_ldf(L.lut + (ch * 256 + y) * 4);
    }
}

// A: the lane's 4 pixels of one output row of the A record, as 12 bytes of HWC BGR (the contrast
// pass-1 arithmetic: resize -> brightness/saturation -> hue), added to the lane's channel sums.
// FAST: every record of the launch has brightness/saturation in the 10-bit fixed point or none, and
// its hue shift, if any, through Bands' SPEC_BS_HUE packed form (hue_pack_n); GENERIC: any photometric
// form (bs_apply's three paths, hue_apply_n).  Two kernels: the generic form's registers would spill
// the fast one's.
struct RecA {
    int      col[4];
    uint32_t wx[4];
    BsRegs   bs;
    int      bs_kind, photo, flip;
};
template <bool FAST>
__device__ __forceinline__ u32x3 rec_pixels(const RecA& R, const RecLds& L, i32x4 ytr, uint32_t& s0, uint32_t& s1,
                                            uint32_t& s2)
{
    const auto sdv  = lds_ptr<const i32x2>(L.hsv);
    const auto hdiv = lds_ptr<const int32_t>(L.hsv + 256 * 8);
    int        val[4][3];
#pragma unroll
    for (int k = 0; k < 4; k++) resize_px<RESIZE_LINEAR, false>(ytr, R.col[k], R.wx[k], val[k]);
    if (R.photo & PHOTO_BS) {
#pragma unroll
        for (int k = 0; k < 4; k++) bs_apply(FAST ? (int)BS_FIXPT : R.bs_kind, R.bs, val[k][0], val[k][1], val[k][2]);
    }
    u32x3 q;
    if (FAST && (R.photo & PHOTO_HUE)) {
        const auto htab8 = lds_ptr<const i32x2>(L.htab) + 30;
        uint32_t   pk[4];
#if AEON_REC_HUE4
        hue_pack_n<4, 0>(sdv, hdiv, htab8, val, pk);
#else
        hue_pack_n<2, 0>(sdv, hdiv, htab8, val, pk);
        hue_pack_n<2, 2>(sdv, hdiv, htab8, val, pk);
#endif
        q = (u32x3){__builtin_amdgcn_perm(pk[1], pk[0], 0x04020100u), __builtin_amdgcn_perm(pk[2], pk[1], 0x05040201u),
                    __builtin_amdgcn_perm(pk[3], pk[2], 0x06050402u)};
    } else {
        if (!FAST && (R.photo & PHOTO_HUE)) {
            const auto htab = lds_ptr<const f32x4>(L.htab) + 30;
            hue_apply_n<2, 0>(sdv, hdiv, htab, val);
            hue_apply_n<2, 2>(sdv, hdiv, htab, val);
        }
        q = (u32x3){(uint32_t)val[0][0] | ((uint32_t)val[0][1] << 8) | ((uint32_t)val[0][2] << 16) | ((uint32_t)val[1][0] << 24),
                    (uint32_t)val[1][1] | ((uint32_t)val[1][2] << 8) | ((uint32_t)val[2][0] << 16) | ((uint32_t)val[2][1] << 24),
                    (uint32_t)val[2][2] | ((uint32_t)val[3][0] << 8) | ((uint32_t)val[3][1] << 16) | ((uint32_t)val[3][2] << 24)};
    }
    // exact channel sums as byte picks of the three words (B0 G0 R0 B1 | G1 R1 B2 G2 | R2 B3 G3 R3)
    s0 = __builtin_amdgcn_udot4(q.x, 0x01000001u, s0, false);
    s0 = __builtin_amdgcn_udot4(q.y, 0x00010000u, s0, false);
    s0 = __builtin_amdgcn_udot4(q.z, 0x00000100u, s0, false);
    s1 = __builtin_amdgcn_udot4(q.x, 0x00000100u, s1, false);
    s1 = __builtin_amdgcn_udot4(q.y, 0x01000001u, s1, false);
    s1 = __builtin_amdgcn_udot4(q.z, 0x00010000u, s1, false);
    s2 = __builtin_amdgcn_udot4(q.x, 0x00010000u, s2, false);
    s2 = __builtin_amdgcn_udot4(q.y, 0x00000100u, s2, false);
    s2 = __builtin_amdgcn_udot4(q.z, 0x01000001u, s2, false);
    return q;
}

// B: the lane's 4 pixels of one output row of the B record from its 12 held bytes, through the
// record table, as one float4 per output plane.
__device__ __forceinline__ void rec_store(const RecLds& L, __amdgpu_buffer_rsrc_t orsrc, int plane, int idx, bool bgr,
                                          uint32_t w0, uint32_t w1, uint32_t w2)
{
    const auto t = [&](int c, uint32_t w, int b) { return lds_ldf(L.rtab + c * 1024 + (int)((w >> (8 * b)) & 0xff) * 4); };
    // channel c of pixel k is byte 3k + c of (w0, w1, w2)
    store_f32x4(orsrc, ((bgr ? 2 : 0) * plane + idx) * 4, t(0, w0, 0), t(0, w0, 3), t(0, w1, 2), t(0, w2, 1));
    __builtin_amdgcn_sched_barrier(0);
    store_f32x4(orsrc, (plane + idx) * 4, t(1, w0, 1), t(1, w1, 0), t(1, w1, 3), t(1, w2, 2));
    __builtin_amdgcn_sched_barrier(0);
    store_f32x4(orsrc, ((bgr ? 0 : 2) * plane + idx) * 4, t(2, w0, 2), t(2, w1, 1), t(2, w2, 0), t(2, w2, 3));
}


// FAST form, A and B of one row of the tile interleaved in one instruction stream: B's table lookups
// of one output plane are issued ahead of a third of A's arithmetic and its float4 store after it,
// so the lookups' LDS latency is covered by A's VALU work instead of stalling every wave of the
// workgroup at once (the waves leave each tile barrier together).  B's stores go through `orsrc`
// with out-of-range offsets (dropped by the buffer bounds check) for lanes without a B row and
// when the step has no B record (its resource has 0 bytes); A's bytes count only where `va`.
__device__ __forceinline__ u32x3 rec_row_fast(const RecA& R, const RecLds& L, i32x4 ytr, bool va, uint32_t& s0,
                                              uint32_t& s1, uint32_t& s2, __amdgpu_buffer_rsrc_t orsrc, int plane,
                                              int idx_b, bool bgr, uint32_t w0, uint32_t w1, uint32_t w2)
{
    const auto T   = [&](int c, uint32_t w, int b) { return lds_ldf(L.rtab + c * 1024 + (int)((w >> (8 * b)) & 0xff) * 4); };
    const auto off = [&](int oc) { return idx_b < 0 ? (int)kOutOfRange : (oc * plane + idx_b) * 4; };
    const auto sdv  = lds_ptr<const i32x2>(L.hsv);
    const auto hdiv = lds_ptr<const int32_t>(L.hsv + 256 * 8);
    const auto htab8 = lds_ptr<const i32x2>(L.htab) + 30;
    // B plane of source channel 0: lookups
    float b[4] = {T(0, w0, 0), T(0, w0, 3), T(0, w1, 2), T(0, w2, 1)};
    __builtin_amdgcn_sched_barrier(0);
    int val[4][3];
#if AEON_REC_HOIST
    resize4_linear<false>(ytr, R.col, R.wx, val); // (the 16 staged words in flight together)
#else
#pragma unroll
    for (int k = 0; k < 4; k++) resize_px<RESIZE_LINEAR, false>(ytr, R.col[k], R.wx[k], val[k]);
#endif
    __builtin_amdgcn_sched_barrier(0);
    store_f32x4(orsrc, off(bgr ? 2 : 0), b[0], b[1], b[2], b[3]);
    float g[4] = {T(1, w0, 1), T(1, w1, 0), T(1, w1, 3), T(1, w2, 2)};
    __builtin_amdgcn_sched_barrier(0);
    if (R.photo & PHOTO_BS) {
#pragma unroll
        for (int k = 0; k < 4; k++) bs_apply(BS_FIXPT, R.bs, val[k][0], val[k][1], val[k][2]);
    }
    uint32_t pk[4];
    const bool hue = (R.photo & PHOTO_HUE) != 0;
    if (hue) hue_pack_n<2, 0>(sdv, hdiv, htab8, val, pk);
    __builtin_amdgcn_sched_barrier(0);
    store_f32x4(orsrc, off(1), g[0], g[1], g[2], g[3]);
    float r[4] = {T(2, w0, 2), T(2, w1, 1), T(2, w2, 0), T(2, w2, 3)};
    __builtin_amdgcn_sched_barrier(0);
    u32x3 q;
    if (hue) {
        hue_pack_n<2, 2>(sdv, hdiv, htab8, val, pk);
        q = (u32x3){__builtin_amdgcn_perm(pk[1], pk[0], 0x04020100u), __builtin_amdgcn_perm(pk[2], pk[1], 0x05040201u),
                    __builtin_amdgcn_perm(pk[3], pk[2], 0x06050402u)};
    } else {
        q = (u32x3){(uint32_t)val[0][0] | ((uint32_t)val[0][1] << 8) | ((uint32_t)val[0][2] << 16) | ((uint32_t)val[1][0] << 24),
                    (uint32_t)val[1][1] | ((uint32_t)val[1][2] << 8) | ((uint32_t)val[2][0] << 16) | ((uint32_t)val[2][1] << 24),
                    (uint32_t)val[2][2] | ((uint32_t)val[3][0] << 8) | ((uint32_t)val[3][1] << 16) | ((uint32_t)val[3][2] << 24)};
    }
    if (!va) q = (u32x3){0u, 0u, 0u};
    s0 = __builtin_amdgcn_udot4(q.x, 0x01000001u, s0, false);
    s0 = __builtin_amdgcn_udot4(q.y, 0x00010000u, s0, false);
    s0 = __builtin_amdgcn_udot4(q.z, 0x00000100u, s0, false);
    s1 = __builtin_amdgcn_udot4(q.x, 0x00000100u, s1, false);
    s1 = __builtin_amdgcn_udot4(q.y, 0x01000001u, s1, false);
    s1 = __builtin_amdgcn_udot4(q.z, 0x00010000u, s1, false);
    s2 = __builtin_amdgcn_udot4(q.x, 0x00010000u, s2, false);
    s2 = __builtin_amdgcn_udot4(q.y, 0x00000100u, s2, false);
    s2 = __builtin_amdgcn_udot4(q.z, 0x01000001u, s2, false);
    __builtin_amdgcn_sched_barrier(0);
    store_f32x4(orsrc, off(bgr ? 0 : 2), r[0], r[1], r[2], r[3]);
    return q;
}

} // namespace

// Development builds (-DAEON_HIP_TRACE, tools/trace_records.py): s_memtime stamps per (workgroup,
// step*8 + tile, slot) -- slots 0..7 by lane 0 of wave 0 (of the first helper wave in the split
// kernel), 16 + w by lane 0 of wave w; entry 63 holds s_memrealtime / s_memtime at entry (0, 1) and
// exit (2, 3).  The product library compiles them out.  (Vector stores: they count on vmcnt, and a
// counted wait that sees more operations after its loads than it assumed only waits longer.)
#ifdef AEON_HIP_TRACE
#define REC_TRACE_SETUP                                                                                      \
    auto stamp = [&](int idx, int sl) {                                                                      \
        if (a.trace && (tid & 63) == 0 && wave == kTraceWave && idx < 64)                                    \
            a.trace[(blockIdx.x * 64 + idx) * 32 + sl] = (uint32_t)__builtin_amdgcn_s_memtime();              \
    };                                                                                                       \
    auto wstamp = [&](int idx) {                                                                             \
        if (a.trace && (tid & 63) == 0 && idx < 64)                                                          \
            a.trace[(blockIdx.x * 64 + idx) * 32 + 16 + wave] = (uint32_t)__builtin_amdgcn_s_memtime();       \
    };                                                                                                       \
    if (a.trace && tid == 0) {                                                                               \
        a.trace[(blockIdx.x * 64 + 63) * 32 + 0] = (uint32_t)__builtin_amdgcn_s_memrealtime();               \
        a.trace[(blockIdx.x * 64 + 63) * 32 + 1] = (uint32_t)__builtin_amdgcn_s_memtime();                   \
    }                                                                                                        \
    if (a.trace && (tid & 63) == 0) /* HW_ID: SIMD id in bits 5:4 */                                         \
        a.trace[(blockIdx.x * 64 + 62) * 32 + 16 + wave] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
#define REC_TRACE_EXIT                                                                                       \
    if (a.trace && tid == 0) {                                                                               \
        a.trace[(blockIdx.x * 64 + 63) * 32 + 2] = (uint32_t)__builtin_amdgcn_s_memrealtime();               \
        a.trace[(blockIdx.x * 64 + 63) * 32 + 3] = (uint32_t)__builtin_amdgcn_s_memtime();                   \
    }
#else
#define REC_TRACE_SETUP                                                                                      \
    auto stamp  = [](int, int) {};                                                                           \
    auto wstamp = [](int) {};
#define REC_TRACE_EXIT
#endif

// One persistent workgroup per CU; records blockIdx.x, +G, ...  Lane (lph, lcg): column group lcg
// (output columns 4*lcg ..), rows lph + 16 j.  Requires every record 3-channel, INTER_LINEAR without
// OpenCV's scalar tail, float32 CHW output through the record table, equal win_w x win_h (host).
template <bool FAST>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) void contrast_records(LaunchArgs a, RecArgs r)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem != 0u) { // see lds_ld
        if (threadIdx.x == 0) atomicOr(a.error, 4);
        return;
    }
    const int    tid = threadIdx.x, nt = blockDim.x;
    const int    wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
    const int    W = r.win_w, H = r.win_h, TS = r.tiles;
    const RecLds L = rec_lds_layout(W, a.stage_bytes);
    const int    gpr = W >> 2;
    const int    lph = tid / gpr, lcg = tid - lph * gpr;
    const int    nph = r.phases, TR = nph * kRecTileRows;
    const bool   active = lph < nph;
    [[maybe_unused]] constexpr int kTraceWave = 0;
    const int    ox0 = lcg * 4;
    const int    plane = W * H;
    const bool   bgr = a.bgr_to_rgb != 0;
    const int    G = gridDim.x;
    const int    K = r.n_jobs > (int)blockIdx.x ? (r.n_jobs - 1 - (int)blockIdx.x) / G + 1 : 0; // this workgroup's records
    if (K == 0) return;
    const auto slot = [&](int k) { return L.job + (k % 3) * (int)sizeof(AugJob); };
    const auto rec_of = [&](int k) { return (int)blockIdx.x + k * G; };
    REC_TRACE_SETUP

    hsv_div_tables(LdsLayout{0, L.hsv, 0, 0, 0, 0, 0, 0, 0, 0}, a.hsv_tables);
    // the launch's constant tables in LDS: the per-record tables are then built without global loads,
    // whose vmcnt waits would drain the B stores in flight at every record boundary
    for (int i = tid; i < 3 * 256; i += nt) lds_ptr<float>(L.lut)[i] = a.lut[i];
    for (int i = tid; i < 256 * 4; i += nt) lds_ptr<int32_t>(L.hwt)[i] = a.hsv_tables[kHsvDivWords + i];
    if (wave == 0) {
        rec_fetch_job(a, rec_of(0), slot(0));
        if (K > 1) rec_fetch_job(a, rec_of(1), slot(1));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    rec_record_tables(a, L, JobRef{slot(0)}, W, FAST);
    // the first tile's staging and row taps
    RecTile f = rec_tile(JobRef{slot(0)}, 0, TR, H, L.stage_bytes, a.error);
    if (f.ok) {
        stage_issue(JobRef{slot(0)}, f.G, L.stage, wave, nw);
        rec_row_taps(JobRef{slot(0)}, f, L.yt, L.stage, tid, nt);
    }
    int pending = 0; // this wave's vector-memory ops issued after its latest staging loads

    uint32_t rec[kRecWords];
#pragma unroll
    for (int i = 0; i < kRecWords; i++) rec[i] = 0;
    uint64_t b_out = 0; // the B record's output item
    int      par   = 0; // staging buffer of the current tile

    for (int k = 0; k <= K; k++) {
        const bool hasA = k < K, hasB = k > 0;
        const JobRef JA{slot(k)};
        RecA R{};
        if (hasA) {
            R.photo   = JF(JA, photo);
            R.bs_kind = JF(JA, bs_kind);
            R.flip    = JF(JA, flip);
            if (R.photo & PHOTO_BS) R.bs = bs_regs(JA);
        }
        const auto orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)b_out, (short)0, hasB ? plane * 12 : 0, 0x00020000);
        uint32_t   s0 = 0, s1 = 0, s2 = 0;
#pragma unroll 1
        for (int t = 0; t < kRecTiles; t++) {
            const bool tile_a = hasA && t < TS; // A has staged rows in this tile
            stamp(k * 8 + t, 0);
            if (tile_a && f.ok) {
                // this wave's staging loads of the tile, then unpack its slots in place
                wait_vm_upto(pending);
                stamp(k * 8 + t, 1);
                stage_unpack(JA, f.G, L.stage + par * L.stage_bytes, wave, nw);
            }
            stamp(k * 8 + t, 2);
            lds_barrier();
            stamp(k * 8 + t, 3);
            if (tile_a && active) { // the lane's column taps (flip folded in) from the record's table
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int   ox  = min(ox0 + q, W - 1);
                    const int   x   = R.flip ? W - 1 - ox : ox;
                    const i32x2 xtt = lds_ptr<const i32x2>(L.xt)[x];
                    R.col[q] = xtt.x, R.wx[q] = (uint32_t)xtt.y;
                }
            }
            // the next tile's staging (this record's next tile, or the next record's first) into the
            // other buffer, and its row taps; the job three records ahead into the freed ring slot
            const bool next_same = hasA && t + 1 < TS;
            const bool next_rec  = hasA && t + 1 == TS && k + 1 < K;
            RecTile    fn{};
            fn.ok = false;
            if (next_same || next_rec) {
                const JobRef JN{slot(next_same ? k : k + 1)};
                if (next_rec && wave == 0 && k + 2 < K) rec_fetch_job(a, rec_of(k + 2), slot(k + 2));
                fn = rec_tile(JN, next_same ? t + 1 : 0, TR, H, L.stage_bytes, a.error);
                if (fn.ok) {
                    const int sb = L.stage + (par ^ 1) * L.stage_bytes;
                    stage_issue(JN, fn.G, sb, wave, nw);
                    pending = 0; // (the counted wait of that tile: the stores issued after these loads)
                    rec_row_taps(JN, fn, L.yt + (par ^ 1) * kRecTRMax * 16, sb, tid, nt);
                }
            }
            stamp(k * 8 + t, 4);
            // the tile's two rows per lane: B's from the oldest held tile, A's into the newest
            uint32_t nwv[6];
#pragma unroll
            for (int u = 0; u < kRecTileRows; u++) {
                const int j = t * kRecTileRows + u;
                const int y = lph + nph * j;
                nwv[3 * u] = nwv[3 * u + 1] = nwv[3 * u + 2] = 0;
                if (FAST && AEON_REC_FUSED && tile_a && f.ok) { // (uniform) A and B interleaved
                    const bool  va  = active && y < H;
                    const i32x4 ytr = lds_ptr<const i32x4>(L.yt + par * kRecTRMax * 16)[min(y - t * TR, TR - 1)];
                    const u32x3 q   = rec_row_fast(R, L, ytr, va, s0, s1, s2, orsrc, plane, hasB && va ? y * W + ox0 : -1,
                                                   bgr, rec[3 * u], rec[3 * u + 1], rec[3 * u + 2]);
                    pending += 3;
                    rec[3 * u] = q.x, rec[3 * u + 1] = q.y, rec[3 * u + 2] = q.z; // (B has read them)
                    continue;
                }
                if (!AEON_REC_NOB && hasB && __builtin_amdgcn_ballot_w64(active && y < H) != 0) {
                    pending += 3;
                    if (active && y < H) rec_store(L, orsrc, plane, y * W + ox0, bgr, rec[3 * u], rec[3 * u + 1], rec[3 * u + 2]);
                }
                if constexpr (!(FAST && AEON_REC_FUSED)) {
                    if (!AEON_REC_NOA && tile_a && f.ok && active && y < H) {
                        const i32x4 ytr = lds_ptr<const i32x4>(L.yt + par * kRecTRMax * 16)[y - t * TR];
                        const u32x3 q   = rec_pixels<FAST>(R, L, ytr, s0, s1, s2);
                        nwv[3 * u] = q.x, nwv[3 * u + 1] = q.y, nwv[3 * u + 2] = q.z;
                    }
                }
            }
            wstamp(k * 8 + t);
            // rotate: drop the tile B consumed, append the tile A produced (the fused rows wrote A's
            // words over B's in place: a cyclic rotation)
            if (FAST && AEON_REC_FUSED && tile_a && f.ok) {
#pragma unroll
                for (int i = 0; i < 6; i++) nwv[i] = rec[i];
            }
#pragma unroll
            for (int i = 0; i < kRecWords - 6; i++) rec[i] = rec[i + 6];
#pragma unroll
            for (int i = 0; i < 6; i++) rec[kRecWords - 6 + i] = nwv[i];
            if (tile_a) par ^= 1;
            if (next_same || next_rec) f = fn; // (the tile staged next; kept through A-less tiles)
        }
        if (!hasA) break;
        // record k is complete in registers: its sums -> (1-c)*mean -> its table; the next record's
        // column taps and hue table
        stamp(k * 8 + 7, 0);
        s0 = wave_sum(s0), s1 = wave_sum(s1), s2 = wave_sum(s2);
        if ((tid & 63) == 0) {
            const auto ps = lds_ptr<uint32_t>(L.sums);
            ps[wave * 4] = s0, ps[wave * 4 + 1] = s1, ps[wave * 4 + 2] = s2;
        }
        lds_barrier(); // also: every lane is done with this step's tiles (B's record table reads)
        stamp(k * 8 + 7, 1);
        rec_table(a, L, JA, W, H, nw, L.sums);
        stamp(k * 8 + 7, 2);
        b_out = JF(JA, out_ptr);
        if (k + 1 < K) rec_record_tables(a, L, JobRef{slot(k + 1)}, W, FAST);
        stamp(k * 8 + 7, 3);
        // (published by the next step's first barrier)
    }
    REC_TRACE_EXIT
}

// The split form (host: AEON_HIP_REC_HELPERS, default): the workgroup's nwc compute waves hold the
// record and do only rows and record ends; nh = blockDim/64 - nwc helper waves (2 for 224-wide
// records: 1,024 lanes) do all of the staging -- job fetches, the next tile's LDS-DMA loads and row
// taps, and, once their loads landed, its in-place unpack -- during the current tile.  The compute
// waves then never wait on a load or unpack, and the helpers run on the issue slots the 14 compute
// waves leave free (they sit 4/4/3/3 on the CU's SIMDs).  The two roles are separate loops (the
// helpers' staging registers are not live across the compute waves' held record) meeting at the same
// barriers: one per tile (B1) and one per record end (B2).
template <bool FAST>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) void contrast_records_split(LaunchArgs a, RecArgs r)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem != 0u) { // see lds_ld
        if (threadIdx.x == 0) atomicOr(a.error, 4);
        return;
    }
    const int    tid = threadIdx.x, nt = blockDim.x;
    const int    wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
    const int    W = r.win_w, H = r.win_h, TS = r.tiles;
    const RecLds L = rec_lds_layout(W, a.stage_bytes);
    const int    gpr = W >> 2;
    const int    nph = r.phases, TR = nph * kRecTileRows;
    const int    nwc = (nph * gpr + 63) >> 6; // compute waves
    const int    nh  = nw - nwc;               // helper waves (>= 1: the host guarantees it)
    const bool   helper = wave >= nwc;
    const int    G = gridDim.x;
    const int    K = r.n_jobs > (int)blockIdx.x ? (r.n_jobs - 1 - (int)blockIdx.x) / G + 1 : 0; // this workgroup's records
    if (K == 0) return;
    const auto slot   = [&](int k) { return L.job + (k % 3) * (int)sizeof(AugJob); };
    const auto rec_of = [&](int k) { return (int)blockIdx.x + k * G; };
    const auto flags  = lds_ptr<int32_t>(L.flags);
    [[maybe_unused]] const int kTraceWave = nwc; // (trace builds: the phase stamps come from the first helper)
    REC_TRACE_SETUP

    // The prologue: each helper fetches the first record's job itself (the same bytes into the same slot)
    // and issues the first tile's staging at once, while the compute waves copy the launch's tables;
    // the helpers unpack after the barrier that publishes the job and the tables.
    if (helper) {
        rec_fetch_job(a, rec_of(0), slot(0));
        if (wave == nwc && K > 1) rec_fetch_job(a, rec_of(1), slot(1));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid - nwc * 64 < 6) lds_ptr<uint32_t>(L.sums)[(tid - nwc * 64) / 3 * 4 + (tid - nwc * 64) % 3] = 0;
    } else {
        hsv_div_tables(LdsLayout{0, L.hsv, 0, 0, 0, 0, 0, 0, 0, 0}, a.hsv_tables);
        for (int i = tid; i < 3 * 256; i += nwc * 64) lds_ptr<float>(L.lut)[i] = a.lut[i];
        for (int i = tid; i < 256 * 4; i += nwc * 64) lds_ptr<int32_t>(L.hwt)[i] = a.hsv_tables[kHsvDivWords + i];
    }
    RecTile f0{};
    if (helper) {
        f0 = rec_tile(JobRef{slot(0)}, 0, TR, H, L.stage_bytes, a.error);
        if (f0.ok) {
            stage_issue(JobRef{slot(0)}, f0.G, L.stage, wave - nwc, nh);
            rec_row_taps(JobRef{slot(0)}, f0, L.yt, L.stage, tid - nwc * 64, nh * 64);
        }
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_barrier();
    rec_record_tables(a, L, JobRef{slot(0)}, W, FAST);

    if (helper) {
        // ---- helpers: stage tile by tile, one tile ahead of the compute waves ----
        const int sw = wave - nwc, stid = tid - nwc * 64, snt = nh * 64;
        // The helpers run at a raised priority: the CU's arbiter otherwise serves the oldest waves first,
        // and the helpers (the youngest) would get issue slots only when the compute waves on their SIMDs
        // stall -- their staging then ends after the compute waves' rows.
        __builtin_amdgcn_s_setprio(AEON_REC_HELPER_PRIO);
        int cur_idx = 0; // (trace builds: the entry the staging stamps go to)
        // (the job's hot half in scalar registers at once: an LDS round trip per field, each waited for,
        // made the helpers' staging the tile's critical path)
        const auto stage_tile = [&](const JobRef& JR, int band, int buf) {
            const JobS    J = job_load(JR.lds);
            const RecTile f = rec_tile(J, band, TR, H, L.stage_bytes, a.error);
            if (f.ok) {
                const int sb = L.stage + buf * L.stage_bytes;
                stage_issue(J, f.G, sb, sw, nh);
                rec_row_taps(J, f, L.yt + buf * kRecTRMax * 16, sb, stid, snt);
                stamp(cur_idx, 5);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // (helpers store nothing)
                stamp(cur_idx, 6);
                stage_unpack(J, f.G, sb, sw, nh);
                stamp(cur_idx, 7);
            }
            if (stid == 0) flags[buf] = f.ok ? 1 : 0;
        };
        int par = 0;
        if (f0.ok) { // the first tile: its loads were issued in the prologue
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            stage_unpack(JobRef{slot(0)}, f0.G, L.stage, sw, nh);
        }
        if (stid == 0) flags[0] = f0.ok ? 1 : 0;
        for (int k = 0; k <= K; k++) {
            const bool hasA = k < K;
#pragma unroll 1
            for (int t = 0; t < kRecTiles; t++) {
                const bool tile_a = hasA && t < TS;
                stamp(k * 8 + t, 0);
                lds_barrier(); // B1: the staged tile is published; the other buffer is free
                stamp(k * 8 + t, 3);
                if (t == 0 && stid < 3) lds_ptr<uint32_t>(L.sums + ((k + 1) & 1) * 16)[stid] = 0; // (see B2)
                const bool next_same = hasA && t + 1 < TS;
                const bool next_rec  = hasA && t + 1 == TS && k + 1 < K;
                cur_idx = k * 8 + t;
                if (next_same || next_rec) {
                    if (next_rec && wave == nwc && k + 2 < K) rec_fetch_job(a, rec_of(k + 2), slot(k + 2));
                    stage_tile(JobRef{slot(next_same ? k : k + 1)}, next_same ? t + 1 : 0, par ^ 1);
                }
                stamp(k * 8 + t, 4);
                wstamp(k * 8 + t);
                if (tile_a) par ^= 1;
            }
            if (!hasA) break;
            stamp(k * 8 + 7, 0);
            lds_barrier(); // B2: the compute waves' sums are in
            stamp(k * 8 + 7, 1);
            rec_table(a, L, JobRef{slot(k)}, W, H, 1, L.sums + (k & 1) * 16);
            stamp(k * 8 + 7, 2);
            if (k + 1 < K) rec_record_tables(a, L, JobRef{slot(k + 1)}, W, FAST);
            stamp(k * 8 + 7, 3);
        }
        REC_TRACE_EXIT
        return;
    }

    // ---- compute waves: rows (A of record k and B of record k - 1), record ends ----
    // The tile loop is unrolled (AEON_REC_UNROLL): tile t's rows live in rec[6t .. 6t + 5] for every
    // record -- B of record k - 1 reads them and A of record k writes them back in place -- so every
    // register index is a compile-time constant without rotating the held record by one tile per tile
    // (42 moves per tile).
    const int  gid = tid; // (compute lanes are the first nwc * 64)
    const int  lph = gid / gpr, lcg = gid - lph * gpr;
    const bool active = lph < nph;
    const int  ox0 = lcg * 4;
    const int  plane = W * H;
    const bool bgr = a.bgr_to_rgb != 0;
    uint32_t   rec[kRecWords];
#pragma unroll
    for (int i = 0; i < kRecWords; i++) rec[i] = 0;
    uint64_t b_out = 0;
    int      par   = 0;
    // the lane's first output row and its index in a plane: every row's y and index are these plus a
    // uniform multiple of nph (computed per row).  Made opaque at each record so that the compiler does
    // not hoist the 14 per-row indices of the unrolled tile loop out of the record loop -- held across
    // it they spilled, and each scratch reload's vmcnt(0) drained the B stores in flight.
    int        lrow = lph, lidx = lph * W + ox0;
    const int  rstep = nph * W;
    for (int k = 0; k <= K; k++) {
        asm volatile("" : "+v"(lrow), "+v"(lidx));
        const bool   hasA = k < K, hasB = k > 0;
        const JobRef JA{slot(k)};
        RecA         R{};
        if (hasA) {
            R.photo   = JF(JA, photo);
            R.bs_kind = JF(JA, bs_kind);
            R.flip    = JF(JA, flip);
            if (R.photo & PHOTO_BS) R.bs = bs_regs(JA);
        }
        const auto orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)b_out, (short)0, hasB ? plane * 12 : 0, 0x00020000);
        uint32_t   s0 = 0, s1 = 0, s2 = 0;
        constexpr bool kUnroll = FAST && AEON_REC_UNROLL; // (the generic form's registers would spill)
#pragma unroll kUnroll ? kRecTiles : 1
        for (int t = 0; t < kRecTiles; t++) {
            const int  rb     = kUnroll ? 6 * t : 0; // the tile's words in rec[]
            const bool tile_a = hasA && t < TS;
            lds_barrier(); // B1
            const bool fok = tile_a && __builtin_amdgcn_readfirstlane(flags[par]) != 0;
            if (tile_a && active) {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int   ox  = min(ox0 + q, W - 1);
                    const int   x   = R.flip ? W - 1 - ox : ox;
                    const i32x2 xtt = lds_ptr<const i32x2>(L.xt)[x];
                    R.col[q] = xtt.x, R.wx[q] = (uint32_t)xtt.y;
                }
            }
            uint32_t nwv[6];
#pragma unroll
            for (int u = 0; u < kRecTileRows; u++) {
                const int j = t * kRecTileRows + u;
                const int y = lrow + nph * j, yi = lidx + rstep * j; // (yi = y * W + ox0)
                uint32_t* hw = rec + rb + 3 * u;
                nwv[3 * u] = nwv[3 * u + 1] = nwv[3 * u + 2] = 0;
                if (FAST && AEON_REC_FUSED && fok) { // (uniform) A and B interleaved
                    const bool  va  = active && y < H;
                    const i32x4 ytr = lds_ptr<const i32x4>(L.yt + par * kRecTRMax * 16)[min(y - t * TR, TR - 1)];
                    const u32x3 q   = rec_row_fast(R, L, ytr, va, s0, s1, s2, orsrc, plane, hasB && va ? yi : -1,
                                                   bgr, hw[0], hw[1], hw[2]);
                    hw[0] = q.x, hw[1] = q.y, hw[2] = q.z; // (B has read them)
                    nwv[3 * u] = q.x, nwv[3 * u + 1] = q.y, nwv[3 * u + 2] = q.z;
                    continue;
                }
                if (hasB && __builtin_amdgcn_ballot_w64(active && y < H) != 0) {
                    if (active && y < H) rec_store(L, orsrc, plane, yi, bgr, hw[0], hw[1], hw[2]);
                }
                if constexpr (!(FAST && AEON_REC_FUSED)) {
                    if (fok && active && y < H) {
                        const i32x4 ytr = lds_ptr<const i32x4>(L.yt + par * kRecTRMax * 16)[y - t * TR];
                        const u32x3 q   = rec_pixels<FAST>(R, L, ytr, s0, s1, s2);
                        nwv[3 * u] = q.x, nwv[3 * u + 1] = q.y, nwv[3 * u + 2] = q.z;
                    }
                }
            }
            wstamp(k * 8 + t);
            if (kUnroll) { // the tile's words: A's (zero where A wrote nothing)
#pragma unroll
                for (int i = 0; i < 6; i++) rec[rb + i] = nwv[i];
            } else { // rotate: drop the tile B consumed, append the tile A produced
#pragma unroll
                for (int i = 0; i < kRecWords - 6; i++) rec[i] = rec[i + 6];
#pragma unroll
                for (int i = 0; i < 6; i++) rec[kRecWords - 6 + i] = nwv[i];
            }
            if (tile_a) par ^= 1;
        }
        if (!hasA) break;
        // the record's channel sums: one LDS add per wave into this record's set (k & 1; the helpers clear
        // the other set in the next step, after every thread has read it for record k - 1)
        s0 = wave_sum(s0), s1 = wave_sum(s1), s2 = wave_sum(s2);
        if ((tid & 63) == 0) {
            const auto ps = lds_ptr<uint32_t>(L.sums + (k & 1) * 16);
            __atomic_fetch_add(ps, s0, __ATOMIC_RELAXED), __atomic_fetch_add(ps + 1, s1, __ATOMIC_RELAXED),
                __atomic_fetch_add(ps + 2, s2, __ATOMIC_RELAXED);
        }
        lds_barrier(); // B2
        rec_table(a, L, JA, W, H, 1, L.sums + (k & 1) * 16);
        b_out = JF(JA, out_ptr);
        if (k + 1 < K) rec_record_tables(a, L, JobRef{slot(k + 1)}, W, FAST);
    }
    REC_TRACE_EXIT
}

// fast: every record's brightness/saturation is the fixed-point cv::transform (or off) -- rec_pixels
hipError_t launch_contrast_records(bool fast, bool split, const LaunchArgs& a, const RecArgs& r, int grid, hipStream_t stream,
                                   hipEvent_t start, hipEvent_t stop)
{
    const void* fn = split ? (fast ? (const void*)contrast_records_split<true> : (const void*)contrast_records_split<false>)
                           : (fast ? (const void*)contrast_records<true> : (const void*)contrast_records<false>);
    void*       args[2] = {(void*)&a, (void*)&r};
    if (start || stop) return hipExtLaunchKernel(fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream, start, stop, 0);
    return hipLaunchKernel(fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream);
}

hipError_t contrast_records_lds_limit(int bytes)
{
    for (const void* fn : {(const void*)contrast_records<true>, (const void*)contrast_records<false>,
                           (const void*)contrast_records_split<true>, (const void*)contrast_records_split<false>}) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

int contrast_records_lds(int win_w, int stage_bytes) { return rec_lds_layout(win_w, stage_bytes).total; }

} // namespace aeon_hip
