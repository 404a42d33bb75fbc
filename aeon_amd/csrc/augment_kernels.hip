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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "augment_device.hpp"
#include "mask16_device.hpp"

namespace aeon_hip {

enum OutForm : int { OF_F32_CHW_VEC = 0, OF_GENERIC = 1 };

#ifndef AEON_HIP_INFO_JOBS // 1: a tile's geometry derived from the job's hot half in SGPRs (0: per-field LDS reads)
#define AEON_HIP_INFO_JOBS 1
#endif

// ---- the band kernel -----------------------------------------------------------------------
// A launch covers n_jobs x max_tiles tiles: tile t = band (t % max_tiles) of job (t / max_tiles),
// a band being TR consecutive output rows of the job's window.  Workgroups are persistent (the
// host sizes the grid to what the CUs hold at once) and take tiles blockIdx.x, +gridDim.x, ...
// for the static rounds, the last rounds from a counter (dynamic tail).  Per tile, one LDS
// staging buffer: LDS-DMA of the tile's source rows + row / column tap tables -> wait -> unpack
// own slots -> barrier -> compute and store -> barrier; the CU's other workgroups cover the
// staging latency, one wave derives the next tile's geometry during the compute.
// A workgroup = 256..512 lanes holding whole 4-pixel column groups of the window (448 = 8 x 56
// for 224-wide outputs); a lane keeps the same four output columns for the whole tile, so their
// resize taps, LDS byte offsets, flip and scalar-tail masks stay in registers, and writes each
// output plane row segment with one 16-byte store per channel.
// KM: KM_FINAL (full record -> loader output), KM_STATS (contrast pass 1: resize + brightness/
// saturation + hue into an HWC uint8 intermediate + exact per-(tile, wave) channel sums), KM_RAW
// (resize only, HWC uint8: the pre-passes).  RM: ResizeMode of every job in the launch.  PHOTO:
// the launch's jobs carry photometric work.  OF: output form (OF_F32_CHW_VEC = float32 CHW planes,
// win_w % 4 == 0, 16-byte aligned items: the ImageNet configuration).  TAIL: some LINEAR job of the
// launch has OpenCV scalar-tail columns (3*dst_w not covered by the SIMD loops).


template <int KM, int RM, bool PHOTO, int OF, bool TAIL>
struct Bands {
    const LaunchArgs& a;
    const LdsLayout&  L;
    int               wave, nw;

    // uniform: tile t -> (job, band) with work, and its staged-source geometry
    struct Info {
        bool      ok;
        int       job, band, y0, nrows;
        int       jl;   // LDS byte address of the job's copy
        int       t;    // the launch tile (-1: no more tiles for this workgroup)
        StageGeom G;
    };
    __device__ __forceinline__ JobRef jref(const Info& f) const { return JobRef{f.jl}; }
    // tile t -> Info; jl: the LDS slot holding the tile's job
    __device__ __forceinline__ Info info(int t, int jl) const
    {
        Info f;
        f.ok   = false;
        f.t    = t;
        f.job  = t / a.max_tiles;
        f.band = t - f.job * a.max_tiles;
        f.jl   = jl;
        // (the job's hot half read at once into scalar registers: the derivation below is on the critical
        // path of the first tile and of every dynamic-tail tile, and each field's LDS round trip was
        // waited for before the next)
#if AEON_HIP_INFO_JOBS
        const JobS J = job_load(jl);
#else
        const JobRef J = jref(f);
#endif
        if (f.band >= JF(J, tiles)) return f;
        if (KM == KM_STATS && JF(J, stats_slot) < 0) return f;
        const int TR = a.rows_per_tile;
        f.y0         = f.band * TR;
        f.nrows      = min(TR, JF(J, win_h) - f.y0);
        if (f.nrows <= 0) return f;
        // source columns (taps are monotone in dx)
        const XTap xf      = xcoef<RM>(JF(J, win_x), JF(J, scale_x), JF(J, crop_w));
        const XTap xl      = xcoef<RM>(JF(J, win_x) + JF(J, win_w) - 1, JF(J, scale_x), JF(J, crop_w));
        const int  two_tap = (RM == RESIZE_LINEAR || RM == RESIZE_AREA2X) ? 1 : 0;
        StageGeom& G       = f.G;
        G.u_lo  = xf.sx;
        G.nc    = xl.sx + two_tap - G.u_lo + 1;
        G.ng    = (G.nc + 3) >> 2;
        G.pitch = 4 * G.ng;
        G.v_lo  = ycoef<RM>(JF(J, win_y) + f.y0, JF(J, scale_y), JF(J, crop_h)).r0;
        G.nr    = ycoef<RM>(JF(J, win_y) + f.y0 + f.nrows - 1, JF(J, scale_y), JF(J, crop_h)).r1 - G.v_lo + 1;
        stage_layout(JF(J, cn), G);
        const int need = stage_need(G, JF(J, cn));
        if (need > L.stage_bytes || JF(J, win_w) > a.max_win_w || f.nrows <= 0) {
            if ((threadIdx.x & 63) == 0) atomicOr(a.error, 2); // (lane 0 of whichever wave derives it)
            return f;
        }
        f.ok = true;
        return f;
    }

    // The next tile's Info through LDS: derived by one wave (its f64 tap bounds are uniform
    // work every wave would otherwise repeat) while the tile before it is computed.
    __device__ __forceinline__ void put_info(const Info& f) const
    {
        if ((threadIdx.x & 63) != 0) return;
        const auto p = lds_ptr<int32_t>(L.info);
        p[0] = f.ok, p[1] = f.job, p[2] = f.band, p[3] = f.y0, p[4] = f.nrows;
        p[5] = f.G.v_lo, p[6] = f.G.nr, p[7] = f.G.u_lo, p[8] = f.G.nc, p[9] = f.G.ng, p[10] = f.G.pitch;
        p[11] = f.G.rp, p[12] = f.t, p[13] = f.jl;
    }
    __device__ __forceinline__ Info get_info() const
    {
        const auto p  = lds_ptr<const int32_t>(L.info);
        const auto rf = [&](int i) { return __builtin_amdgcn_readfirstlane(p[i]); };
        Info       f;
        f.ok = rf(0) != 0, f.job = rf(1), f.band = rf(2), f.y0 = rf(3), f.nrows = rf(4);
        f.G.v_lo = rf(5), f.G.nr = rf(6), f.G.u_lo = rf(7), f.G.nc = rf(8), f.G.ng = rf(9), f.G.pitch = rf(10);
        f.G.rp = rf(11), f.t = rf(12), f.jl = rf(13);
        return f;
    }

    // Issue the tile's LDS-DMA staging (loads in flight on return).
    __device__ __forceinline__ void issue(const Info& f) const
    {
        if (f.ok) stage_issue(jref(f), f.G, L.stage, wave, nw);
    }
    // The tile's row taps; its column taps and hue table too unless the LDS still holds this
    // record's (build_xt / build_rec false: the workgroup's previous tile was of the same record).
    __device__ __forceinline__ void tables(const Info& f, bool build_xt, bool build_rec = true) const
    {
        if (!f.ok) return;
        const JobRef J = jref(f);
        const StageGeom& G = f.G;
        const int  stage = L.stage;
        const int  tid = threadIdx.x, nt = blockDim.x;
        if (build_xt) {
            const auto xt = lds_ptr<i32x2>(L.xt);
            for (int x = tid; x < JF(J, win_w); x += nt) {
                const XTap c = xcoef<RM>(JF(J, win_x) + x, JF(J, scale_x), JF(J, crop_w));
                xt[x]        = (i32x2){4 * (c.sx - G.u_lo), (c.a0 & 0xffff) | (c.a1 << 16)};
            }
        }
        if (PHOTO && KM != KM_RAW && a.has_hue && build_rec && JF(J, cn) == 3 && (JF(J, photo) & PHOTO_HUE)) {
            // the record's hue table (kHueTabBytes): cvtColor's H of h12, + hue, % 180 as uchar
            const int     tab = L.hsv + kHsvLdsDivBytes;
            const f32x4*  wt  = reinterpret_cast<const f32x4*>(a.hsv_tables + kHsvDivWords);
            const int     hue = JF(J, hue);
            const bool    sp  = fast_photo(f);
            for (int i = tid; i < kHueTabEntries; i += nt) {
                const int   h12 = i - 30;
                const f32x4 w   = wt[(((h12 < 0 ? h12 + 180 : h12) + hue) % 180) & 0xff];
                if (!sp) {
                    lds_ptr<f32x4>(tab)[i] = w;
                    continue;
                }
                // hue_pack_n's entry: a channel with w == 0 takes v (byte 0), another with w == 1
                // takes t1 (byte 1), the third t_w (byte 2) with its w
                const int iv = w[0] == 0.f ? 0 : (w[1] == 0.f ? 1 : 2);
                int       i1 = -1;
                for (int c = 0; c < 3; c++)
                    if (c != iv && i1 < 0 && w[c] == 1.f) i1 = c;
                if (i1 < 0) i1 = iv == 0 ? 1 : 0, atomicOr(a.error, 16); // impossible (every sector has t1)
                const int iw  = 3 - iv - i1;
                uint32_t  sel = 0x0c000000u;
                for (int c = 0; c < 3; c++) sel |= (uint32_t)(c == iv ? 0 : (c == i1 ? 1 : 2)) << (8 * c);
                lds_ptr<i32x2>(tab)[i] = (i32x2){(int)__float_as_uint(w[iw]), (int)sel};
            }
        }
        const auto yt = lds_ptr<i32x4>(L.yt);
        for (int r = tid; r < f.nrows; r += nt) {
            const YTap y = ycoef<RM>(JF(J, win_y) + f.y0 + r, JF(J, scale_y), JF(J, crop_h));
            yt[r]        = (i32x4){stage + (y.r0 - G.v_lo) * G.rp, stage + (y.r1 - G.v_lo) * G.rp, y.b0, y.b1};
        }
    }

    // The per-channel tail of the record's chain -- contrast -> lighting -> standardize, each a
    // function of one u8 channel value (image.cpp:336-346, 398-405, etl_image.cpp:316-339) -- as one
    // 3 x 256 f32 table in LDS for the tile's record, so the pixel loop does one lookup per channel.
    __device__ __forceinline__ bool uses_rtab(const JobRef& J) const
    {
        return KM == KM_FINAL && PHOTO && a.has_rtab && JF(J, cn) == 3 && (JF(J, photo) & (PHOTO_CONTRAST | PHOTO_LIGHTING));
    }
    // lds_shifts: the record's (1-c)*mean per channel in LDS (null: from a.shifts, contrast_reduce's)
    __device__ __forceinline__ void record_table(const Info& f,
                                                 const __attribute__((address_space(3))) double* lds_shifts = nullptr) const
    {
        if (!f.ok) return;
        const JobRef J = jref(f);
        if (!uses_rtab(J)) return;
        const int photo = JF(J, photo);
        double    sh[3] = {0, 0, 0};
        if ((photo & PHOTO_CONTRAST) && lds_shifts) {
            sh[0] = lds_shifts[0], sh[1] = lds_shifts[1], sh[2] = lds_shifts[2];
        } else if (photo & PHOTO_CONTRAST) {
            const double* p = a.shifts + (size_t)JF(J, stats_slot) * 4;
            sh[0] = p[0], sh[1] = p[1], sh[2] = p[2];
        }
        const float c = JF(J, contrast), la = JF(J, light_a);
        const auto  rt = lds_ptr<float>(L.rtab);
        for (int i = threadIdx.x; i < 3 * 256; i += blockDim.x) {
            const int ch = i >> 8;
            int       y  = i & 255;
            if (photo & PHOTO_CONTRAST) y = u8rnd((float)((double)((float)y * c + 0.f) + sh[ch]));
            if (photo & PHOTO_LIGHTING) y = sat_u8(u8rnd((float)y * la + 0.f) + JFA(J, light_add, ch));
            rt[i] = lut_at(ch, y << 2);
        }
    }

    __device__ __forceinline__ void unpack(const Info& f) const
    {
        if (f.ok) stage_unpack(jref(f), f.G, L.stage, wave, nw);
    }

    // SPEC_BS_HUE: the tile's record is known (fast_photo) to be 3-channel, 4-pixel-aligned, with
    // brightness/saturation in the 10-bit fixed-point cv::transform and a hue shift:
    // the pixel loop then carries no per-pixel branches on those run-time choices (their merged
    // paths cost ~7 VALU per pixel: conversions and moves the compiler hoists out of the branches).
    enum : int { SPEC_NONE = 0, SPEC_BS_HUE = 1 };
    static constexpr bool kHasSpec = KM == KM_STATS && PHOTO && RM == RESIZE_LINEAR && !TAIL;
    __device__ __forceinline__ bool fast_photo(const Info& f) const
    {
        if (!kHasSpec || !f.ok) return false;
        const JobRef J = jref(f);
        return JF(J, cn) == 3 && (JF(J, photo) & (PHOTO_BS | PHOTO_HUE)) == (PHOTO_BS | PHOTO_HUE) && JF(J, bs_kind) == BS_FIXPT &&
               (JF(J, win_w) & 3) == 0;
    }
    __device__ __forceinline__ int compute_any(const Info& f) const
    {
        if constexpr (kHasSpec)
            if (fast_photo(f)) return compute<SPEC_BS_HUE>(f);
        return compute<SPEC_NONE>(f);
    }

    // Compute and store tile t from buffer b.  Returns a lower bound on the vector-memory
    // instructions this wave issued (its stores): all younger than the next tile's staging loads.
    template <int SPEC = SPEC_NONE>
    __device__ __forceinline__ int compute(const Info& f) const
    {
        if (!f.ok) return 0;
        constexpr bool SP = SPEC == SPEC_BS_HUE;
        const int  band = f.band, y0 = f.y0, nrows = f.nrows;
        const JobRef J = jref(f);
        const int  tid   = threadIdx.x;
        const int  nt    = blockDim.x;
        const int  cn    = SP ? 3 : JF(J, cn);
        const int  win_w = JF(J, win_w);
        const auto xt    = lds_ptr<const i32x2>(L.xt);
        const auto yt    = lds_ptr<const i32x4>(L.yt);
        const auto sdv   = lds_ptr<const i32x2>(L.hsv);
        const auto hdiv  = lds_ptr<const int32_t>(L.hsv + 256 * 8);
        // (a STATS tile's chain ends at the intermediate: only BS and HUE matter to it)
        const int  photo = SP ? (PHOTO_BS | PHOTO_HUE) : (PHOTO && KM != KM_RAW && cn == 3) ? JF(J, photo) : 0;
        double     sh0 = 0, sh1 = 0, sh2 = 0;
        if (KM == KM_FINAL && (photo & PHOTO_CONTRAST)) {
            const double* sh = a.shifts + (size_t)JF(J, stats_slot) * 4;
            sh0 = sh[0], sh1 = sh[1], sh2 = sh[2];
        }
        uint32_t sum0 = 0, sum1 = 0, sum2 = 0;
        const auto htab  = lds_ptr<const f32x4>(L.hsv + kHsvLdsDivBytes) + 30; // at h12 = 0
        const auto htab8 = lds_ptr<const i32x2>(L.hsv + kHsvLdsDivBytes) + 30; // SPEC_BS_HUE form
        BsRegs   bsr{};
        int      bs_kind = 0;
        if (PHOTO && (photo & PHOTO_BS)) bs_kind = SP ? (int)BS_FIXPT : JF(J, bs_kind), bsr = bs_regs(J);

        const int  elem  = KM != KM_FINAL ? 1 : out_elem_bytes(a.out_dtype);
        const int  plane = win_w * JF(J, win_h);
        const int  obytes = (KM == KM_FINAL ? JF(J, out_plane) : plane) * cn * elem;
        const auto orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)JF(J, out_ptr), (short)0, obytes, 0x00020000);
        const bool tail  = TAIL && RM == RESIZE_LINEAR && JF(J, xv) < JF(J, dst_w) * cn; // OpenCV scalar row tail
        const int  wx0   = JF(J, win_x);
        const int  xv    = JF(J, xv);
        const int  flip  = JF(J, flip);
        const int  bgr   = a.bgr_to_rgb && cn == 3;
        // Lane -> (column group, row phase), fixed for the tile
        const int  gpr    = (win_w + 3) >> 2;
        const bool full4  = SP || (win_w & 3) == 0; // every lane's group is 4 pixels of the window
        const int  ncg    = min(gpr, nt);
        const int  nph    = nt / ncg;
        const int  lph    = tid / ncg;
        const int  lcg    = tid - lph * ncg;
        const bool active = lph < nph;
        // values carried from the resize to the store: 4x scaled (see resize_px) unless photometric
        constexpr bool SC = !PHOTO;
        const bool     rtab = uses_rtab(J);
        auto lut_of = [&](int c, int v) { return rtab ? lds_ldf(L.rtab + (c * 256 + v) * 4) : lut_at(c, SC ? v : v << 2); };
        auto u8_of  = [&](int v) { return SC ? v >> 2 : v; };
        // uint8 output value of source channel c: the plain byte, or its fixed_aspect_ratio
        // uint8 standardize through the LUT
        auto u8_out = [&](int c, int v) { return a.u8_map ? (int)lut_of(c, v) : u8_of(v); };

        for (int cg = active ? lcg : gpr; cg < gpr; cg += ncg) {
            const int ox0 = cg * 4;
            const int nk  = SP ? 4 : min(4, win_w - ox0);
            int       col[4];
            uint32_t  wxk[4];
            int       tmask = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                // columns past the window edge recompute the last one (never stored)
                const int  ox  = min(ox0 + k, win_w - 1);
                const int  x   = flip ? win_w - 1 - ox : ox;
                const i32x2 xtt = xt[x];
                col[k]         = xtt.x; // byte offset in a staged row
                wxk[k]         = (uint32_t)xtt.y;
                if (TAIL && RM == RESIZE_LINEAR && tail && (wx0 + x) * cn + 2 >= xv) tmask |= 1 << k;
            }
            for (int ry = lph; ry < nrows; ry += nph) {
                const i32x4 ytr = yt[ry];
                const int   y   = y0 + ry; // window row
                int         val[4][3];
#pragma unroll
                for (int k = 0; k < 4; k++) {
#ifdef AEON_HIP_EXP_NORESIZE // development ablation: no gathers / resize math (wrong values)
                    val[k][0] = ytr.x + col[k], val[k][1] = ytr.y + col[k], val[k][2] = ytr.z + (int)wxk[k];
#else
                    resize_px<RM, SC>(ytr, col[k], wxk[k], val[k]);
#endif
                }
                if (TAIL && RM == RESIZE_LINEAR && tmask) {
#pragma unroll
                    for (int k = 0; k < 4; k++)
                        if (tmask & (1 << k)) {
                            const int ox = min(ox0 + k, win_w - 1);
                            const int x  = flip ? win_w - 1 - ox : ox;
                            tail_fix<SC>(ytr, col[k], wxk[k], (wx0 + x) * cn, xv, val[k]);
                        }
                }
                if constexpr (SP) {
                    // fixed-point brightness/saturation -> hue, packed (B, G, R, 0) per pixel ->
                    // exact channel sums (v_dot4 byte picks) -> 12 bytes of HWC uint8
#pragma unroll
                    for (int k = 0; k < 4; k++) bs_apply(BS_FIXPT, bsr, val[k][0], val[k][1], val[k][2]);
                    uint32_t pk[4];
#if AEON_HIP_HUE_PACK4
                    hue_pack_n<4, 0>(sdv, hdiv, htab8, val, pk);
#else
                    hue_pack_n<2, 0>(sdv, hdiv, htab8, val, pk);
                    hue_pack_n<2, 2>(sdv, hdiv, htab8, val, pk);
#endif
                    // the 12-byte HWC group B0 G0 R0 B1 | G1 R1 B2 G2 | R2 B3 G3 R3, and the exact channel
                    // sums as byte picks of those three words (9 v_dot4 instead of 12 on the pixels)
                    const u32x3 q = {__builtin_amdgcn_perm(pk[1], pk[0], 0x04020100u),
                                     __builtin_amdgcn_perm(pk[2], pk[1], 0x05040201u),
                                     __builtin_amdgcn_perm(pk[3], pk[2], 0x06050402u)};
                    sum0 = __builtin_amdgcn_udot4(q.x, 0x01000001u, sum0, false);
                    sum0 = __builtin_amdgcn_udot4(q.y, 0x00010000u, sum0, false);
                    sum0 = __builtin_amdgcn_udot4(q.z, 0x00000100u, sum0, false);
                    sum1 = __builtin_amdgcn_udot4(q.x, 0x00000100u, sum1, false);
                    sum1 = __builtin_amdgcn_udot4(q.y, 0x01000001u, sum1, false);
                    sum1 = __builtin_amdgcn_udot4(q.z, 0x00010000u, sum1, false);
                    sum2 = __builtin_amdgcn_udot4(q.x, 0x00010000u, sum2, false);
                    sum2 = __builtin_amdgcn_udot4(q.y, 0x00000100u, sum2, false);
                    sum2 = __builtin_amdgcn_udot4(q.z, 0x01000001u, sum2, false);
                    __builtin_amdgcn_raw_buffer_store_b96(q, orsrc, (y * win_w + ox0) * 3, 0, 0);
                    continue;
                }
                if (PHOTO && photo) {
#ifndef AEON_HIP_EXP_NOBS // development ablation: no brightness/saturation (wrong values)
                    if (photo & PHOTO_BS) {
#pragma unroll
                        for (int k = 0; k < 4; k++) bs_apply(bs_kind, bsr, val[k][0], val[k][1], val[k][2]);
                    }
#endif
#ifdef AEON_HIP_EXP_NOHUE // development ablation: no hue (wrong values)
                    if (false) {
#else
                    if (photo & PHOTO_HUE) {
#endif // two pixels at a time: four cost 14 VGPRs (a wave per SIMD)
                        hue_apply_n<kHueBatch, 0>(sdv, hdiv, htab, val);
                        if (kHueBatch < 4) hue_apply_n<kHueBatch, kHueBatch % 4>(sdv, hdiv, htab, val);
                        if (kHueBatch == 1) {
                            hue_apply_n<1, 2>(sdv, hdiv, htab, val);
                            hue_apply_n<1, 3>(sdv, hdiv, htab, val);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        int bb = val[k][0], gg = val[k][1], rr = val[k][2];
                        if (KM == KM_STATS) { // the intermediate keeps the post-hue pixel
                            if (full4 || k < nk) sum0 += bb, sum1 += gg, sum2 += rr;
                            val[k][0] = bb, val[k][1] = gg, val[k][2] = rr;
                            continue;
                        }
                        if (rtab) { // contrast / lighting folded into the record table
                            val[k][0] = bb, val[k][1] = gg, val[k][2] = rr;
                            continue;
                        }
                        if (photo & PHOTO_CONTRAST) {
                            const float c = JF(J, contrast);
                            bb = u8rnd((float)((double)((float)bb * c + 0.f) + sh0));
                            gg = u8rnd((float)((double)((float)gg * c + 0.f) + sh1));
                            rr = u8rnd((float)((double)((float)rr * c + 0.f) + sh2));
                        }
                        if (photo & PHOTO_LIGHTING) {
                            const float la = JF(J, light_a);
                            bb = sat_u8(u8rnd((float)bb * la + 0.f) + JFA(J, light_add, 0));
                            gg = sat_u8(u8rnd((float)gg * la + 0.f) + JFA(J, light_add, 1));
                            rr = sat_u8(u8rnd((float)rr * la + 0.f) + JFA(J, light_add, 2));
                        }
                        val[k][0] = bb, val[k][1] = gg, val[k][2] = rr;
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
#ifdef AEON_HIP_EXP_NOSTORE // development ablation: no output stores
                        if (lut_of(c, val[0][c]) == 1234.5f)
#endif
                        store_f32x4(orsrc, (oc * plane + idx) * 4, lut_of(c, val[0][c]), lut_of(c, val[1][c]),
                                    lut_of(c, val[2][c]), lut_of(c, val[3][c]));
                        // one channel's four LUT reads in flight at a time: hoisting all twelve
                        // costs ~20 VGPRs (two waves per SIMD) for no measurable overlap
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    continue;
                }
                if (a.out_dtype == OUT_U8 && (a.channel_major || cn == 1) && nk == 4) {
                    // uint8 planes (pixel masks, uint8 images): a lane's 4 consecutive output
                    // bytes of a plane as one dword store when the 4-byte group is aligned
#pragma unroll
                    for (int c = 0; c < 3; c++) {
                        if (c >= cn) break;
                        const int oc = bgr ? 2 - c : c;
                        const int i0 = (cn == 1 ? 0 : oc * JF(J, out_plane)) + y * JF(J, out_pitch) + ox0;
                        const uint32_t w = ((uint32_t)u8_out(c, val[0][c]) & 0xff) | (((uint32_t)u8_out(c, val[1][c]) & 0xff) << 8) |
                                           (((uint32_t)u8_out(c, val[2][c]) & 0xff) << 16) | ((uint32_t)u8_out(c, val[3][c]) << 24);
                        if ((i0 & 3) == 0) {
                            __builtin_amdgcn_raw_buffer_store_b32(w, orsrc, i0, 0, kStoreAux);
                        } else {
#pragma unroll
                            for (int k = 0; k < 4; k++)
                                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w >> (8 * k)), orsrc, i0 + k, 0, kStoreAux);
                        }
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
                        const int i = a.channel_major ? oc * JF(J, out_plane) + y * JF(J, out_pitch) + ox0 + k
                                                      : (y * JF(J, out_pitch) + ox0 + k) * cn + oc;
                        // image::loader (convert_mix_channels: Mat::convertTo of the uint8 record,
                        // saturating; standardize for float / double)
                        const int v = u8_of(val[k][c]);
                        switch (a.out_dtype) {
                        case OUT_F32:
                            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(lut_of(c, val[k][c])), orsrc, i * 4, 0,
                                                                  kStoreAux);
                            break;
                        case OUT_F64: { // CV_64F standardize: every op in double (image.cpp:129-174)
                            double d = (double)v;
                            if (a.has_mean) {
                                d = d * (1. / 255.) - a.smean[c];
                                if (a.sinv[c] != 0) d = d * a.sinv[c];
                            }
                            const uint64_t bits = __double_as_longlong(d);
                            __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)bits, (uint32_t)(bits >> 32)}, orsrc,
                                                                  i * 8, 0, kStoreAux);
                            break;
                        }
                        case OUT_S8:
                            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)min(v, 127), orsrc, i, 0, kStoreAux);
                            break;
                        case OUT_S16:
                        case OUT_U16:
                            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, orsrc, i * 2, 0, kStoreAux);
                            break;
                        case OUT_S32:
                            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, orsrc, i * 4, 0, kStoreAux);
                            break;
                        default:
                            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)u8_out(c, val[k][c]), orsrc, i, 0, kStoreAux);
                        }
                    }
                }
            }
        }

        if (KM == KM_STATS) { // exact per-(tile, wave) sums; unused wave slots are zeroed
            sum0 = wave_sum(sum0), sum1 = wave_sum(sum1), sum2 = wave_sum(sum2);
            const int lane = tid & 63;
            uint32_t* p    = a.partials + ((size_t)JF(J, stats_slot) * a.partial_stride + (size_t)band * 8) * 4;
            auto put = [&](uint32_t* q, uint32_t v) { *q = v; };
            if (lane == 0) put(p + wave * 4 + 0, sum0), put(p + wave * 4 + 1, sum1), put(p + wave * 4 + 2, sum2);
            if (wave == 0 && lane >= nw && lane < 8) put(p + lane * 4 + 0, 0), put(p + lane * 4 + 1, 0), put(p + lane * 4 + 2, 0);
        }
        // stores per wave when every lane is busy on whole rows of whole 4-pixel groups (one row
        // set of nrows / nph rows per lane): 3 per row for float32 planes, 1 (a 12-byte group)
        // for the HWC uint8 intermediates; otherwise 0 (the caller then drains everything)
        const bool regular = ncg == gpr && nt % ncg == 0 && (win_w & 3) == 0 && nrows % nph == 0;
        const int  per_row = (KM == KM_FINAL && OF == OF_F32_CHW_VEC) ? 3 : ((KM != KM_FINAL && cn == 3) ? 1 : 0);
        return regular ? per_row * (nrows / nph) : 0;
    }
};

// The contrast pass 1 with photometric stages (VALU-bound) is held to 80 VGPRs: 6 waves per SIMD =
// three 512-lane workgroups per CU (at 85 VGPRs it gets two).
template <int KM, int RM, bool PHOTO, int OF, bool TAIL>
#ifndef AEON_HIP_STATS_MIN_WAVES
#define AEON_HIP_STATS_MIN_WAVES 6
#endif
// Contrast pass 2 (the photometric copy pass, 512-lane workgroups) likewise: at 82 VGPRs it held
// two workgroups per CU, at 80 three (C3 pass 2 131-132 -> 127 us).
#ifndef AEON_HIP_PASS2_MIN_WAVES
#define AEON_HIP_PASS2_MIN_WAVES 6
#endif
constexpr int kMinWaves = (KM == KM_STATS && PHOTO && !TAIL) ? AEON_HIP_STATS_MIN_WAVES
                          : (KM == KM_FINAL && RM == RESIZE_COPY && PHOTO) ? AEON_HIP_PASS2_MIN_WAVES
                                                                          : AEON_HIP_MIN_WAVES;

// An image + mask call in one launch: after its last tile, every workgroup draws the masks' NEAREST
// row blocks (nearest_staged's work: row map, source-row copy, gather; mask16_device.hpp) from a
// counter until it runs dry -- exactly m_blocks + G draws, the last of which resets the counter -- so
// the masks fill the image tiles' ragged end instead of a launch of their own.  8-bit masks to uint8
// outputs (the host's condition).  Written lean (job fields uniform, 16 output columns per lane as 8
// VGPRs of perm selectors or packed columns) so that the form keeps the tile kernel's occupancy.  LDS
// from a.m_lds: the row map, the block's job, the draw word, then the staged rows (m_slots x m_pitch
// bytes); the tiles' staging buffer is free by then.
__device__ __forceinline__ uint32_t lds_word_u(const char* p) { return __builtin_amdgcn_readfirstlane(*(const uint32_t*)p); }

__device__ __forceinline__ void mask_gather_u8(const Mask16Job& J, const RowMap& M, int pitch, const uint8_t* lds, bool perm_ok)
{
    constexpr int C   = 16; // output columns per lane
    const int     tid = threadIdx.x;
    const int     ng  = (J.out_w + C - 1) / C;
    const int     per = min(ng, (int)blockDim.x), rstep = blockDim.x / per, r0 = tid / per;
    if (r0 >= rstep) return;
    const uint32_t* lds32 = (const uint32_t*)lds;
    auto col = [&](int x) { // source column of output column x (cv::flip after the resize)
        const int dx = J.flip ? J.out_w - 1 - x : x;
        return min((int)floor(dx * J.scale_x), J.crop_w - 1);
    };
    for (int g = tid % per; g < ng; g += per) {
        const int x0 = g * C;
        const int nk = min(C, J.out_w - x0);
        int       lo[4];
        uint32_t  rel[4];
        bool      ok = perm_ok && nk == C && ((J.out_ptr + (size_t)M.y0 * J.out_pitch + x0) & 15) == 0 && (J.out_pitch & 15) == 0;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            int c[4];
#pragma unroll
            for (int k = 0; k < 4; k++) c[k] = col(min(x0 + 4 * w + k, J.out_w - 1));
            lo[w]  = min(c[0], c[3]); // ascending, or descending when flipped
            ok     = ok && max(c[0], c[3]) - lo[w] <= 4;
            rel[w] = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) rel[w] |= (uint32_t)(c[k] - lo[w]) << (8 * k); // (fallback: <= 255 apart)
        }
        if (ok) { // every 4 outputs from 5 consecutive staged bytes: one read pair + one v_perm_b32
            for (int r = r0; r < M.nrows; r += rstep) {
                const int s    = M.slot[r];
                const int rowb = s * pitch + (int)(seg_start(J, M, s) & 15);
                u32x4     q;
#pragma unroll
                for (int w = 0; w < 4; w++) {
                    const int      at  = rowb + lo[w];
                    const uint32_t sel = rel[w] + (uint32_t)(at & 3) * 0x01010101u;
                    q[w]               = __builtin_amdgcn_perm(lds32[(at >> 2) + 1], lds32[at >> 2], sel);
                }
                __builtin_nontemporal_store(q, gptr<u32x4>(J.out_ptr + (size_t)(M.y0 + r) * J.out_pitch + x0));
            }
            continue;
        }
        // otherwise element by element (downscales beyond 4/3 across, unaligned rows, the last group)
        for (int r = r0; r < M.nrows; r += rstep) {
            const int      s    = M.slot[r];
            const uint8_t* base = lds + s * pitch + (int)(seg_start(J, M, s) & 15);
            const uint64_t dst  = J.out_ptr + (size_t)(M.y0 + r) * J.out_pitch + x0;
            for (int k = 0; k < nk; k++) gptr<uint8_t>(dst)[k] = base[col(x0 + k)];
        }
    }
}

// Schedule: workgroup b's first block is block b (its job words loaded at kernel entry, `jw`), the
// rest are drawn from the counter (blocks G + c); the next block's draw and job load are issued before
// this block's gather, so neither latency is on the block chain.  A launch with more blocks than
// workgroups draws exactly (blocks - G) + G times (every workgroup ends on one failing draw; the last
// draw resets the counter); with fewer, none.
#ifndef AEON_HIP_MASK_LOADS // 16-byte row loads in flight per lane (the tile kernel's VGPR budget)
#define AEON_HIP_MASK_LOADS 4
#endif
__device__ __forceinline__ uint32_t mask_job_word(const LaunchArgs& a, int k)
{
    const int tid = threadIdx.x;
    if (k < 0 || tid >= (int)(sizeof(Mask16Job) / 4)) return 0;
    return gptr<const uint32_t>((uint64_t)(a.mjobs + k / a.m_bpj))[tid];
}

__device__ __forceinline__ void mask_blocks(const LaunchArgs& a, char* smem, uint32_t jw)
{
    constexpr int kMapBytes = (int)((sizeof(RowMap) + 15) & ~(size_t)15);
    constexpr int kJobBytes = (int)sizeof(Mask16Job);
    static_assert(kJobBytes % 16 == 0 && kJobBytes / 4 <= 64, "Mask16Job: whole 16-byte units, one wave");
    static_assert(kMapBytes + kJobBytes + 16 == kMaskBlockHdrBytes, "mask16.hpp's LDS header size");
    RowMap&        M    = *reinterpret_cast<RowMap*>(smem + a.m_lds);
    char*          jl   = smem + a.m_lds + kMapBytes;
    uint32_t&      draw = *reinterpret_cast<uint32_t*>(smem + a.m_lds + kMapBytes + kJobBytes);
    uint8_t*       rows = reinterpret_cast<uint8_t*>(smem + a.m_lds + kMapBytes + kJobBytes + 16);
    const int      tid  = threadIdx.x;
    const int      G    = gridDim.x;
    const uint32_t D    = a.m_blocks > G ? (uint32_t)(a.m_blocks - G) : 0u; // drawn blocks
    int            k    = (int)blockIdx.x < a.m_blocks ? (int)blockIdx.x : -1;
    uint32_t       nraw = 0;
    if (D && tid == 0) nraw = atomicAdd(a.m_ctr, 1u);
    while (k >= 0) {
        lds_barrier(); // (the tiles' staging buffer / the previous block's rows are free)
        if (tid < kJobBytes / 4) reinterpret_cast<uint32_t*>(jl)[tid] = jw;
        lds_barrier();
        Mask16Job J; // uniform: scalar registers
        {
            uint32_t* w = reinterpret_cast<uint32_t*>(&J);
#pragma unroll
            for (int i = 0; i < kJobBytes / 4; i++) w[i] = lds_word_u(jl + 4 * i);
        }
        const int rec = k / a.m_bpj;
        const int y0  = (k - rec * a.m_bpj) * a.m_rows;
        const bool has = y0 < J.out_h; // (uniform: a mask shorter than the call's tallest has no block here)
        if (has && tid < 64) map_rows(J, rec, y0, min(a.m_rows, J.out_h - y0), a.m_slots, M);
        if (tid == 0) {
            uint32_t c = ~0u;
            if (D) {
                c = nraw;
                if (c == D + G - 1) atomicExch(a.m_ctr, 0u); // the launch's last draw
                if (c > D + G - 1) atomicOr(a.error, 32);    // a counter left over by a launch
            }
            draw = c;
        }
        lds_barrier();
        if (has) copy_rows<AEON_HIP_MASK_LOADS>(J, M, seg_blocks(J), a.m_pitch, rows);
        lds_barrier();
        // the next block: its draw and job load in flight during this block's gather
        const uint32_t c  = __builtin_amdgcn_readfirstlane(draw);
        const int      kn = c < D ? G + (int)c : -1;
        if (kn >= 0) {
            jw = mask_job_word(a, kn);
            if (tid == 0) nraw = atomicAdd(a.m_ctr, 1u);
        }
        if (has) mask_gather_u8(J, M, a.m_pitch, rows, a.m_perm != 0);
        k = kn;
    }
}

// MASKS: the image + mask form (KM_FINAL only): the launch's masks' row blocks after the tiles
template <int KM, int RM, bool PHOTO, int OF, bool TAIL, bool MASKS = false>
__global__ __launch_bounds__(kBlockMax)
__attribute__((amdgpu_waves_per_eu(kMinWaves<KM, RM, PHOTO, OF, TAIL>)))
void augment_tiles(LaunchArgs a)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem != 0u) { // see lds_ld
        if (threadIdx.x == 0) atomicOr(a.error, 4);
        return;
    }
    const int       tid = threadIdx.x, nt = blockDim.x;
    const int       wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
    const LdsLayout L = lds_layout(a.max_win_w, a.rows_per_tile, a.stage_bytes, PHOTO && a.has_hue, a.has_rtab != 0);
    const Bands<KM, RM, PHOTO, OF, TAIL> W{a, L, wave, nw};

    // per-launch tables
#ifndef AEON_HIP_LUT_DMA
#define AEON_HIP_LUT_DMA 1
#endif
    if (KM == KM_FINAL && (a.out_dtype == OUT_F32 || a.u8_map)) {
        if (AEON_HIP_LUT_DMA) {
            // by LDS-DMA, 256 bytes per wave instruction: no VGPR round trip and no wait here, so the
            // loads are in flight together with the first jobs' fetch (one wait for both, below)
            const auto rs = uniform_rsrc((const void*)a.lut, 3 * 256 * 4);
            for (int i = wave; i < 12; i += nw) lds_dma<4>(rs, L.lut + i * 256, (uint32_t)((tid & 63) * 4 + i * 256));
        } else {
            const auto lut = lds_ptr<float>(L.lut);
            for (int i = tid; i < 3 * 256; i += nt) lut[i] = a.lut[i];
        }
    }
    if (PHOTO && KM != KM_RAW && a.has_hue) {
        hsv_div_tables(L, a.hsv_tables);
    }
    // (the record tables read the LUT: the wait + barrier before the first tile orders them)
    // an image + mask launch: the job of this workgroup's first mask block, loaded now
    const uint32_t mjw = MASKS ? mask_job_word(a, (int)blockIdx.x < a.m_blocks ? (int)blockIdx.x : -1) : 0u;
    // development builds (-DAEON_HIP_TRACE, tools/trace_kernel.py): s_memtime stamps per (workgroup,
    // iteration, phase) when a.trace is set; s_memrealtime (chip-wide 100 MHz) at entry and exit.
    // The product library compiles them out.
#ifdef AEON_HIP_TRACE
    auto stamp = [&](int it, int ph) {
        if (a.trace && tid == 0 && it < 16)
            a.trace[(blockIdx.x * 16 + it) * 16 + ph] = (uint32_t)__builtin_amdgcn_s_memtime();
    };
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16) * 16 + 15] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16) * 16 + 14] = (uint32_t)__builtin_amdgcn_s_memtime();
#else
    auto stamp = [](int, int) {};
#endif
    using Info = typename Bands<KM, RM, PHOTO, OF, TAIL>::Info;
    // Schedule: static rounds, tiles blockIdx.x, +G, +2G, ... (the tiles in flight at any moment are
    // consecutive bands of a few records: measured faster than contiguous ranges per workgroup and
    // than a fully counter-fed schedule), then a dynamic tail: the tiles of the partial last round
    // plus tail_rounds full rounds before it go to whichever workgroups finish their static tiles
    // first, one counter draw per tile and one failing draw per workgroup -- exactly t_tail + G draws,
    // the last of which resets the ring slot's counter for its next launch.
    const int T      = a.total_tiles, G = gridDim.x;
    const int t_tail = a.tail_ctr ? min(T % G + a.tail_rounds * G, T - T % G == 0 ? T : T - G) : 0;
    const int t_dyn  = T - t_tail; // first dynamically handed-out tile
    auto draw = [&]() -> int { // the next dynamic tile, or -1
        const auto slot = lds_ptr<uint32_t>(L.info + 60);
        if (tid == 0) {
            const uint32_t k = atomicAdd(a.tail_ctr, 1u);
            if (k == (uint32_t)(t_tail + G - 1)) atomicExch(a.tail_ctr, 0u); // the last draw of the launch
            if (k >= (uint32_t)(t_tail + G)) atomicOr(a.error, 32);        // a counter left over by a launch
            *slot = k;
        }
        __syncthreads();
        const int k = (int)__builtin_amdgcn_readfirstlane(*slot);
        return k < t_tail ? t_dyn + k : -1;
    };
    // Job slots: three, a ring.  A static tile's job is fetched two tiles ahead by wave 0, after its
    // share of the staging loads, so that the wave's staging wait (vmcnt(1)) leaves the fetch in
    // flight (loads and stores retire in order on the vector-memory counter): a job read over PCIe
    // from a pinned host table is not waited for on the critical path.  The next static tile's
    // geometry is derived from its (landed) job by one wave during the compute.  A dynamic-tail tile
    // is drawn when the workgroup gets to it and its job fetched then: drawing a tile ahead (so the
    // fetch could land during the compute) hands out the last tiles a tile's time earlier and
    // lengthened the tail more than the hidden fetch saved (C2 44.8 vs 42.7 us).
    const auto slot_of = [&](int i) { return L.job + (i % 3) * (int)sizeof(AugJob); };
    int  t        = blockIdx.x;
    int  prev_job = -1;
    bool live     = t < t_dyn;
    if (t_tail && !live) { // no static tile: start with a drawn one
        t    = draw();
        live = t >= 0;
    }
    int js = 0; // ring index of the current tile's job slot
    // The prologue waits for the first tile's job only: every workgroup fetches at once (768 x 128 B
    // over PCIe for C2), and the second job is not needed before the first tile's compute, so it is
    // fetched with the first tile's staging loads.
#ifndef AEON_HIP_FETCH1
#define AEON_HIP_FETCH1 1
#endif
    if (wave == 0) {
        fetch_job(a, live ? t : -1, slot_of(0));
        if (!AEON_HIP_FETCH1) fetch_job(a, live && t + G < t_dyn ? t + G : -1, slot_of(1));
    }
    stamp(0, 10);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stamp(0, 11);
    __syncthreads();
    stamp(0, 12);
    Info f{};
    if (live) f = W.info(t, slot_of(0));
    stamp(0, 13);
    for (int it = 0; live; it++) {
        // the staging phases (LDS-DMA issue, tap tables, unpack) at a raised wave priority: they
        // are this workgroup's critical path while the CU's other workgroups stream stores
        // (measured 38.8 -> 37.7 us on C2); the VALU-bound contrast pass 1 prefers the reverse
        // (293 -> 283 us on C3)
        __builtin_amdgcn_s_setprio(KM == KM_STATS ? kComputePrio : kStagePrio);
        stamp(it, 0);
        const bool more  = t + G < t_dyn;     // a static next tile (its job is in slot js + 1)
        const bool more2 = t + 2 * G < t_dyn; // ... and a static one after it
        stamp(it, 1);
        W.issue(f);
        if (AEON_HIP_FETCH1 && it == 0 && wave == 0 && more) fetch_job(a, t + G, slot_of(js + 1));
        if (wave == 0 && more2) fetch_job(a, t + 2 * G, slot_of(js + 2));
        stamp(it, 2);
        const bool same = f.ok && f.job == prev_job; // the LDS tables still hold this record's
        prev_job        = f.ok ? f.job : -1;
        W.tables(f, !same, !same);
        W.record_table(f);
        stamp(it, 3);
        // the staging loads (and in the first tile the next tile's job): all but the newest fetch
        if (wave == 0 && more2) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stamp(it, 4);
        W.unpack(f);
        stamp(it, 5);
        lds_barrier(); // (not __syncthreads: a fence there would wait for wave 0's job fetch)
        stamp(it, 6);
        __builtin_amdgcn_s_setprio(KM == KM_STATS ? kStagePrio : kComputePrio);
        if (more && wave == nw - 1) W.put_info(W.info(t + G, slot_of(js + 1)));
        W.compute_any(f);
        stamp(it, 7);
        lds_barrier(); // everyone is done reading the buffer before it is refilled
        stamp(it, 8);
        if (more) {
            f = W.get_info();
            t += G;
            js = (js + 1) % 3;
        } else if (t_tail) {
            t    = draw();
            live = t >= 0;
            if (live) {
                js = (js + 1) % 3;
                if (wave == 0) fetch_job(a, t, slot_of(js));
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                f = W.info(t, slot_of(js));
            }
        } else {
            break;
        }
    }
    if constexpr (MASKS) mask_blocks(a, smem, mjw);
#ifdef AEON_HIP_TRACE
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16 + 1) * 16 + 15] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
}


// Contrast pass 2 prologue: per stats slot, (1-c)*mean per channel from the exact per-(tile,
// wave) sums of pass 1 (cv::mean = sum * (1./N), kept in f64).  One 64-lane workgroup per job
// of the pass-2 launch.
__global__ __launch_bounds__(64) void contrast_reduce(LaunchArgs a, int n_jobs)
{
    const int job = blockIdx.x;
    if (job >= n_jobs) return;
    cjob& J = job_ref(a, job);
    if (J.stats_slot < 0 || J.cn != 3 || !(J.photo & PHOTO_CONTRAST)) return;
    const int          tid = threadIdx.x;
    unsigned long long s0 = 0, s1 = 0, s2 = 0;
    for (int e = tid; e < J.stats_tiles * 8; e += 64) {
        const uint32_t* p = a.partials + ((size_t)J.stats_slot * a.partial_stride + e) * 4;
        s0 += p[0], s1 += p[1], s2 += p[2];
    }
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_xor(s0, o);
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    if (tid == 0) {
        const double inv_n = 1. / (double)(J.win_w * J.win_h);
        const double k     = 1.0 - (double)J.contrast;
        double*      sh    = a.shifts + (size_t)J.stats_slot * 4;
        sh[0] = k * ((double)s0 * inv_n);
        sh[1] = k * ((double)s1 * inv_n);
        sh[2] = k * ((double)s2 * inv_n);
    }
}

// ---- host-side launch helpers (stage.cpp) ----------------------------------------------------
typedef void (*KernelFn)(LaunchArgs);

template <int KM, int RM, bool TAIL>
KernelFn pick_form(bool photo, int of, bool masks)
{
    if (masks) { // image + mask launches: KM_FINAL
        if constexpr (KM != KM_FINAL || RM == RESIZE_AREA2X) {
            return nullptr;
        } else {
            if (of == OF_F32_CHW_VEC)
                return photo ? augment_tiles<KM, RM, true, OF_F32_CHW_VEC, TAIL, true>
                             : augment_tiles<KM, RM, false, OF_F32_CHW_VEC, TAIL, true>;
            return photo ? augment_tiles<KM, RM, true, OF_GENERIC, TAIL, true> : augment_tiles<KM, RM, false, OF_GENERIC, TAIL, true>;
        }
    }
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
KernelFn pick_rm(int rm, bool tail, bool photo, int of, bool masks)
{
    switch (rm) {
    case RESIZE_LINEAR:
        return tail ? pick_form<KM, RESIZE_LINEAR, true>(photo, of, masks) : pick_form<KM, RESIZE_LINEAR, false>(photo, of, masks);
    case RESIZE_AREA2X: return pick_form<KM, RESIZE_AREA2X, false>(photo, of, masks);
    case RESIZE_NEAREST: return pick_form<KM, RESIZE_NEAREST, false>(photo, of, masks);
    default: return pick_form<KM, RESIZE_COPY, false>(photo, of, masks);
    }
}

KernelFn pick_kernel(int km, int rm, bool tail, bool photo, int of, bool masks = false)
{
    if (km == KM_FINAL) return pick_rm<KM_FINAL>(rm, tail, photo, of, masks);
    if (masks) return nullptr;
    if (km == KM_STATS) return pick_rm<KM_STATS>(rm, tail, true, OF_GENERIC, false);
    return pick_rm<KM_RAW>(rm, tail, false, OF_GENERIC, false);
}

int out_form(const LaunchArgs& a) { return (a.out_dtype == OUT_F32 && a.channel_major && a.vec_ok) ? OF_F32_CHW_VEC : OF_GENERIC; }

// start/stop (optional): events the dispatch itself stamps when the kernel starts and ends
// (hipExtLaunchKernel), i.e. the kernel's own duration -- the same interval rocprofv3 reports --
// with no extra packets between launches.
hipError_t launch_tiles(int km, int rm, bool tail, bool photo, const LaunchArgs& a, int grid, hipStream_t stream,
                        hipEvent_t start, hipEvent_t stop)
{
    const KernelFn fn = pick_kernel(km, rm, tail, photo, out_form(a), a.m_blocks > 0);
    if (!fn) return hipErrorInvalidDeviceFunction;
    if (start || stop) {
        void* args[1] = {(void*)&a};
        return hipExtLaunchKernel((const void*)fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream, start, stop, 0);
    }
    hipLaunchKernelGGL(fn, dim3(grid), dim3(a.threads), a.lds_bytes, stream, a);
    return hipGetLastError();
}

hipError_t launch_contrast_reduce(const LaunchArgs& a, int n_jobs, hipStream_t stream)
{
    hipLaunchKernelGGL(contrast_reduce, dim3(n_jobs), dim3(64), 0, stream, a, n_jobs);
    return hipGetLastError();
}

// Workgroups of this kernel form one CU holds at once (persistent grid sizing).
hipError_t kernel_occupancy(int km, int rm, bool tail, bool photo, const LaunchArgs& a, int* blocks)
{
    const KernelFn fn = pick_kernel(km, rm, tail, photo, out_form(a), a.m_blocks > 0);
    if (!fn) return hipErrorInvalidDeviceFunction;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, (const void*)fn, a.threads, a.lds_bytes);
}

hipError_t set_kernel_lds_limit(int bytes)
{
    for (int km = 0; km < 3; km++)
        for (int rm = 0; rm < 4; rm++)
            for (int ph = 0; ph < 4; ph++)
                for (int of = 0; of < 4; of++) {
                    const KernelFn fn = pick_kernel(km, rm, (ph & 2) != 0, (ph & 1) != 0, of & 1, of >= 2);
                    if (!fn) continue;
                    hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
                    if (e != hipSuccess) return e;
                }
    return hipSuccess;
}

} // namespace aeon_hip
