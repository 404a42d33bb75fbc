// split_kernels.hip -- the single-pass image tile kernel (aeon's transform_single_image + loader::load
// for a record with no photometric stage: crop -> INTER_LINEAR resize -> flip -> BGR->RGB + CHW +
// standardize, /root/reference/src/etl_image.cpp:146-202, 246-341) with its staging taken off the
// waves that store.
//
// augment_tiles (augment_kernels.hip) runs three 448-lane workgroups per CU, each staging a tile and
// then computing it: while a workgroup stages (LDS-DMA issue, wait, unpack, tap tables, ~4 us per
// tile), its waves store nothing, and a CU holds only ~7 tiles of the C2 batch, so the chip's first
// stores start after a whole staging phase and the persistent grid's tail is a tile's latency long.
// Here one 1,024-lane workgroup per CU splits the roles (as contrast_records_split does for C3):
//   * nwc compute waves (16 row phases x 56 column groups = 14 waves for 224-wide windows) only read
//     the staged tile from LDS, resize, standardize through the LUT and stream float4 stores;
//   * the remaining helper waves (2) fetch the jobs, issue the NEXT tile's LDS-DMA into the other of
//     two staging buffers, build its column / row tap tables, wait for their own loads and unpack in
//     place, at raised priority (s_setprio 3), while the compute waves work on the current tile.
// The roles meet at one barrier per tile; the compute waves never wait on a load (their stores stay
// in flight across the barriers: lds_barrier does not drain vmcnt).  Tiles: t = blockIdx.x + k * G
// (interleaved: the tiles in flight at any moment are consecutive bands of consecutive records, so the
// write stream stays one contiguous window of HBM).  Every byte equals augment_tiles' (the arithmetic
// is augment_device.hpp's: resize_px / tail_fix / lut_at), i.e. the oracle's.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "augment_device.hpp"

#ifndef AEON_SPLIT_HELPER_PRIO
#define AEON_SPLIT_HELPER_PRIO 3
#endif

namespace aeon_hip {

namespace {

// The staged geometry of tile t (job in LDS slot jl): uniform.  Mirrors Bands::info for INTER_LINEAR.
struct SplitTile {
    bool      ok;
    int       job, band, y0, nrows;
    StageGeom G;
};
__device__ __forceinline__ SplitTile split_tile(const LaunchArgs& a, const JobRef& J, int t, int TR, int stage_bytes)
{
    SplitTile f;
    f.ok   = false;
    f.job  = t / a.max_tiles;
    f.band = t - f.job * a.max_tiles;
    if (f.band >= JF(J, tiles)) return f;
    f.y0    = f.band * TR;
    f.nrows = min(TR, JF(J, win_h) - f.y0);
    if (f.nrows <= 0) return f;
    const XTap xf = xcoef<RESIZE_LINEAR>(JF(J, win_x), JF(J, scale_x), JF(J, crop_w));
    const XTap xl = xcoef<RESIZE_LINEAR>(JF(J, win_x) + JF(J, win_w) - 1, JF(J, scale_x), JF(J, crop_w));
    StageGeom& G  = f.G;
    G.u_lo        = xf.sx;
    G.nc          = xl.sx + 1 - G.u_lo + 1;
    G.ng          = (G.nc + 3) >> 2;
    G.pitch       = 4 * G.ng;
    G.v_lo        = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0, JF(J, scale_y), JF(J, crop_h)).r0;
    G.nr          = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0 + f.nrows - 1, JF(J, scale_y), JF(J, crop_h)).r1 - G.v_lo + 1;
    stage_layout(3, G);
    if (JF(J, cn) != 3 || stage_need(G, 3) > stage_bytes) {
        if ((threadIdx.x & 63) == 0) atomicOr(a.error, 2);
        return f;
    }
    f.ok = true;
    return f;
}

} // namespace

// Development builds (-DAEON_HIP_TRACE): s_memtime stamps per (workgroup, tile k < 16, slot) into
// a.trace[(blockIdx.x * 16 + k) * 16 + slot]: helper slots 0-5 (stage start, job/geometry, loads issued,
// tables, loads landed, unpacked), compute slots 8-10 (barrier passed, stores issued, -), entry / exit
// s_memrealtime in tile 15's slots 14 / 15.
template <bool TAIL>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4))) void augment_split(LaunchArgs a, SplitArgs s)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem != 0u) { // see lds_ld
        if (threadIdx.x == 0) atomicOr(a.error, 4);
        return;
    }
    const int      tid = threadIdx.x, nt = blockDim.x;
    const int      wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
    const int      nwc = s.nwc, nh = nw - nwc;
    const bool     helper = wave >= nwc;
    const SplitLds L   = split_lds_layout(s.win_w, a.stage_bytes);
    const int      TR  = a.rows_per_tile;
    const int      G   = gridDim.x;
    const int      T   = a.total_tiles;
    const int      K   = T > (int)blockIdx.x ? (T - 1 - (int)blockIdx.x) / G + 1 : 0; // this workgroup's tiles
    if (K == 0) return;
    const auto slot    = [&](int k) { return L.job + (k % kSplitJobs) * (int)sizeof(AugJob); };
    const auto tile_of = [&](int k) { return (int)blockIdx.x + k * G; };
#ifdef AEON_HIP_TRACE
    auto stamp = [&](int k, int sl) {
        if (a.trace && (tid & 63) == 0 && (sl < 8 ? wave == nwc : wave == 0) && k < 16)
            a.trace[(blockIdx.x * 16 + k) * 16 + sl] = (uint32_t)__builtin_amdgcn_s_memtime();
    };
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16 + 15) * 16 + 14] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#else
    auto stamp = [](int, int) {};
#endif

    if (helper) {
        // ---- helpers: tile k + 1 staged while the compute waves work on tile k ----
        const int sw = wave - nwc, stid = tid - nwc * 64, snt = nh * 64;
        __builtin_amdgcn_s_setprio(AEON_SPLIT_HELPER_PRIO);
        // every helper wave fetches the first tile's job itself (the same bytes into the same slot)
        fetch_job(a, tile_of(0), slot(0));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const auto stage = [&](int k) {
            const int    buf = k & 1;
            const JobRef J{slot(k)};
            stamp(k, 0);
            if (sw == 0 && k + 1 < K) fetch_job(a, tile_of(k + 1), slot(k + 1)); // (landed by this stage's wait)
            const SplitTile f  = split_tile(a, J, tile_of(k), TR, L.stage_bytes);
            const int       sb = L.stage + buf * L.stage_bytes;
            stamp(k, 1);
            if (f.ok) {
                stage_issue(J, f.G, sb, sw, nh);
                stamp(k, 2);
                const auto xt = lds_ptr<i32x2>(L.xt + buf * L.xt_bytes);
                for (int x = stid; x < s.win_w; x += snt) {
                    const XTap c = xcoef<RESIZE_LINEAR>(JF(J, win_x) + x, JF(J, scale_x), JF(J, crop_w));
                    xt[x]        = (i32x2){4 * (c.sx - f.G.u_lo), (c.a0 & 0xffff) | (c.a1 << 16)};
                }
                const auto yt = lds_ptr<i32x4>(L.yt + buf * kSplitTRMax * 16);
                for (int r = stid; r < f.nrows; r += snt) {
                    const YTap y = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0 + r, JF(J, scale_y), JF(J, crop_h));
                    yt[r]        = (i32x4){sb + (y.r0 - f.G.v_lo) * f.G.rp, sb + (y.r1 - f.G.v_lo) * f.G.rp, y.b0, y.b1};
                }
            }
            if (stid == 0) {
                const auto p = lds_ptr<int32_t>(L.info + buf * 64);
                p[0] = f.ok ? 1 : 0, p[1] = f.y0, p[2] = f.nrows;
            }
            stamp(k, 3);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // (helpers store nothing)
            stamp(k, 4);
            if (f.ok) stage_unpack(J, f.G, sb, sw, nh);
            stamp(k, 5);
        };
        stage(0);
        lds_barrier(); // B0: tile 0 staged, the LUT in
        for (int k = 0; k < K; k++) {
            if (k + 1 < K) stage(k + 1);
            lds_barrier(); // tile k computed (its buffer free), tile k + 1 staged
        }
#ifdef AEON_HIP_TRACE
        if (a.trace && tid == nwc * 64) a.trace[(blockIdx.x * 16 + 15) * 16 + 15] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
        return;
    }

    // ---- compute waves ----
    {
        const auto rs = uniform_rsrc((const void*)a.lut, 3 * 256 * 4);
        for (int i = wave; i < 12; i += nwc) lds_dma<4>(rs, L.lut + i * 256, (uint32_t)((tid & 63) * 4 + i * 256));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int  W      = s.win_w;
    const int  gpr    = W >> 2;
    const int  nph    = s.nph;
    const int  lph    = tid / gpr, lcg = tid - lph * gpr;
    const bool active = lph < nph;
    const int  ox0    = lcg * 4;
    const bool bgr    = a.bgr_to_rgb != 0;
    lds_barrier(); // B0
    for (int k = 0; k < K; k++) {
        const int  buf  = k & 1;
        const auto info = lds_ptr<const int32_t>(L.info + buf * 64);
        const bool ok   = __builtin_amdgcn_readfirstlane(info[0]) != 0;
        stamp(k, 8);
        if (ok && active) {
            const JobRef J{slot(k)};
            const int    y0 = __builtin_amdgcn_readfirstlane(info[1]), nrows = __builtin_amdgcn_readfirstlane(info[2]);
            const int    H = JF(J, win_h), flip = JF(J, flip);
            const int    plane = W * H;
            const auto   orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)JF(J, out_ptr), (short)0, JF(J, out_plane) * 12, 0x00020000);
            const auto   xt    = lds_ptr<const i32x2>(L.xt + buf * L.xt_bytes);
            const auto   yt    = lds_ptr<const i32x4>(L.yt + buf * kSplitTRMax * 16);
            int          col[4];
            uint32_t     wxk[4];
            int          tmask = 0;
            const int    wx0 = JF(J, win_x), xv = JF(J, xv);
            const bool   tail = TAIL && xv < JF(J, dst_w) * 3;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int   ox  = ox0 + q;
                const int   x   = flip ? W - 1 - ox : ox;
                const i32x2 xtt = xt[x];
                col[q] = xtt.x, wxk[q] = (uint32_t)xtt.y;
                if (TAIL && tail && (wx0 + x) * 3 + 2 >= xv) tmask |= 1 << q;
            }
            for (int ry = lph; ry < nrows; ry += nph) {
                const i32x4 ytr = yt[ry];
                int         val[4][3];
#pragma unroll
                for (int q = 0; q < 4; q++) resize_px<RESIZE_LINEAR, true>(ytr, col[q], wxk[q], val[q]);
                if (TAIL && tmask) {
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        if (tmask & (1 << q)) {
                            const int x = flip ? W - 1 - (ox0 + q) : ox0 + q;
                            tail_fix<true>(ytr, col[q], wxk[q], (wx0 + x) * 3, xv, val[q]);
                        }
                }
                const int idx = (y0 + ry) * W + ox0;
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const int oc = bgr ? 2 - c : c;
                    store_f32x4(orsrc, (oc * plane + idx) * 4, lut_at(c, val[0][c]), lut_at(c, val[1][c]),
                                lut_at(c, val[2][c]), lut_at(c, val[3][c]));
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        stamp(k, 9);
        lds_barrier(); // the buffer of tile k is free; tile k + 1 is staged
    }
}

hipError_t launch_split(bool tail, const LaunchArgs& a, const SplitArgs& s, int grid, hipStream_t stream, hipEvent_t start,
                        hipEvent_t stop)
{
    const void* fn      = tail ? (const void*)augment_split<true> : (const void*)augment_split<false>;
    void*       args[2] = {(void*)&a, (void*)&s};
    if (start || stop) return hipExtLaunchKernel(fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream, start, stop, 0);
    return hipLaunchKernel(fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream);
}

hipError_t split_lds_limit(int bytes)
{
    for (const void* fn : {(const void*)augment_split<true>, (const void*)augment_split<false>}) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

} // namespace aeon_hip
