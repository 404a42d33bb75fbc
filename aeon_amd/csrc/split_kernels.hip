// split_kernels.hip -- the single-pass image tile kernel (aeon's transform_single_image + loader::load
// for a record with no photometric stage: crop -> INTER_LINEAR resize -> flip -> BGR->RGB + CHW +
// standardize, /root/reference/src/etl_image.cpp:146-202, 246-341) with its staging taken off the
// waves that store.
//
// augment_tiles (augment_kernels.hip) runs three 448-lane workgroups per CU, each staging a tile and
// then computing it: while a workgroup stages (LDS-DMA issue, wait, unpack, tap tables, ~4 us per
// tile), its waves store nothing, and a CU holds only ~7 tiles of the C2 batch, so the chip's first
// stores start after a whole staging phase and the persistent grid's tail is a tile's latency long.
// Here one 1,024-lane workgroup per CU runs the tiles as a software pipeline over three LDS staging
// buffers: in the step of tile k every wave issues its share of tile k + 2's LDS-DMA (and the tile's
// column / row tap tables), the compute waves (16 row phases x 56 column groups = 14 waves for 224-wide
// windows) resize, standardize through the LUT and stream float4 stores for tile k, and then every wave
// waits -- counting exactly the operations it issued after them, so its stores stay in flight -- for
// its loads of tile k + 1 and unpacks them in place.  One barrier per tile; a tile's loads have two
// tiles' time to land.  (A form with the staging on two helper waves only, as contrast_records_split
// does for C3, measured 51.7 / 45.5 us with two / three buffers against augment_tiles' 41: two waves
// issue, build tables and unpack a C2 tile in ~5 us, while the compute waves need ~1.8 us.)  Tiles:
// t = blockIdx.x + k * G (interleaved: the tiles in flight at any moment are consecutive bands of
// consecutive records, so the write stream stays one contiguous window of HBM).  Every byte equals
// augment_tiles' (the arithmetic is augment_device.hpp's: resize_px / tail_fix / lut_at), i.e. the
// oracle's.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "augment_device.hpp"

#ifndef AEON_SPLIT_GEO_PRIO
#define AEON_SPLIT_GEO_PRIO 3
#endif

namespace aeon_hip {

namespace {

// The staged geometry of tile t (job in LDS slot jl): uniform.  Mirrors Bands::info for INTER_LINEAR.
struct SplitTile {
    bool      ok;
    int       job, band, y0, nrows;
    StageGeom G;
};
__device__ __forceinline__ SplitTile split_tile(const LaunchArgs& a, const JobS& J, int t, int TR, int stage_bytes)
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

// Wait until at most n vector-memory operations of this wave are outstanding, n exact (an immediate per
// value).  Loads and stores retire in order on the counter, so "the loads issued before the last n
// operations have landed" -- without draining the stores issued since.  n >= 63: the counter cannot hold
// more than 63, so anything issued 63 operations ago has retired already.
__device__ __forceinline__ void wait_vm_exact(int n)
{
    switch (n) {
#define AEON_VM(i) case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
    AEON_VM(0) AEON_VM(1) AEON_VM(2) AEON_VM(3) AEON_VM(4) AEON_VM(5) AEON_VM(6) AEON_VM(7) AEON_VM(8) AEON_VM(9)
    AEON_VM(10) AEON_VM(11) AEON_VM(12) AEON_VM(13) AEON_VM(14) AEON_VM(15) AEON_VM(16) AEON_VM(17) AEON_VM(18)
    AEON_VM(19) AEON_VM(20) AEON_VM(21) AEON_VM(22) AEON_VM(23) AEON_VM(24) AEON_VM(25) AEON_VM(26) AEON_VM(27)
    AEON_VM(28) AEON_VM(29) AEON_VM(30) AEON_VM(31) AEON_VM(32) AEON_VM(33) AEON_VM(34) AEON_VM(35) AEON_VM(36)
    AEON_VM(37) AEON_VM(38) AEON_VM(39) AEON_VM(40) AEON_VM(41) AEON_VM(42) AEON_VM(43) AEON_VM(44) AEON_VM(45)
    AEON_VM(46) AEON_VM(47) AEON_VM(48) AEON_VM(49) AEON_VM(50) AEON_VM(51) AEON_VM(52) AEON_VM(53) AEON_VM(54)
    AEON_VM(55) AEON_VM(56) AEON_VM(57) AEON_VM(58) AEON_VM(59) AEON_VM(60) AEON_VM(61) AEON_VM(62)
#undef AEON_VM
    default:
        if (n < 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        break;
    }
}

// Development builds (-DAEON_HIP_TRACE): s_memtime stamps per (workgroup, tile k < 15, slot) into
// a.trace[(blockIdx.x * 16 + k) * 16 + slot], by lane 0 of the last wave (slots 0-4) and of wave 0 (slots
// 8-12): iteration start (after the barrier), tile k + 2 issued, tile k computed, tile k + 1's loads landed,
// unpacked.  Tile 15's slots 13 / 14 / 15: s_memtime and s_memrealtime at entry, s_memrealtime at exit.
// OCC: workgroups per CU the register budget leaves room for (1: <= 128 VGPRs; 2: <= 64, two 1,024-lane
// workgroups whose phases interleave, each with a third of the CU's LDS or less)
template <bool TAIL, int OCC>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4 * OCC))) void augment_split(LaunchArgs a, SplitArgs s)
{
    extern __shared__ __attribute__((aligned(16))) char smem[];
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem != 0u) { // see lds_ld
        if (threadIdx.x == 0) atomicOr(a.error, 4);
        return;
    }
    const int      tid = threadIdx.x, nt = blockDim.x;
    const int      wave = __builtin_amdgcn_readfirstlane(tid >> 6), nw = nt >> 6;
    const int      lane = tid & 63;
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
        if (a.trace && lane == 0 && (sl < 8 ? wave == nw - 1 : wave == 0) && k < 15)
            a.trace[(blockIdx.x * 16 + k) * 16 + sl] = (uint32_t)__builtin_amdgcn_s_memtime();
    };
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16 + 15) * 16 + 14] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16 + 15) * 16 + 13] = (uint32_t)__builtin_amdgcn_s_memtime();
#else
    auto stamp = [](int, int) {};
#endif
    // the compute lanes: (row phase lph, column group lcg) of the first nph * W / 4 lanes
    const int  W      = s.win_w;
    const int  gpr    = W >> 2;
    const int  nph    = s.nph;
    const int  lph    = tid / gpr, lcg = tid - lph * gpr;
    const bool active = lph < nph;
    const int  ox0    = lcg * 4;
    const bool bgr    = a.bgr_to_rgb != 0;
    // this wave's stores for a full tile: 3 planes x rpl rows when its first lane computes (every compute
    // lane has exactly rpl rows of a tile of TR = nph * rpl rows)
    const int  pmin   = (wave * 64) / gpr;
    const int  s_full = pmin < nph ? 3 * s.rpl : 0;

    // A tile's geometry (split_tile: its band, staged rows and columns -- uniform f64 work) is computed once,
    // by the last wave (it stores nothing), a tile ahead of the issue that needs it, into the geometry ring.
    const auto geo_slot = [&](int k) { return L.info + (k % kSplitGeo) * 64; };
    const auto put_geo  = [&](int k) {
        const SplitTile f = split_tile(a, job_load(slot(k)), tile_of(k), TR, L.stage_bytes);
        if (lane == 0) {
            const auto p = lds_ptr<int32_t>(geo_slot(k));
            p[0] = f.ok ? 1 : 0, p[1] = f.y0, p[2] = f.nrows, p[3] = f.G.v_lo, p[4] = f.G.nr, p[5] = f.G.u_lo;
            p[6] = f.G.nc, p[7] = f.G.ng, p[8] = f.G.pitch, p[9] = f.G.rp;
        }
    };
    const auto get_geo = [&](int k) -> SplitTile {
        const auto p = lds_ptr<const i32x4>(geo_slot(k));
        const i32x4 q0 = p[0], q1 = p[1], q2 = p[2];
        const auto  rf = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
        SplitTile   f;
        f.ok = rf(q0.x) != 0, f.y0 = rf(q0.y), f.nrows = rf(q0.z), f.G.v_lo = rf(q0.w);
        f.G.nr = rf(q1.x), f.G.u_lo = rf(q1.y), f.G.nc = rf(q1.z), f.G.ng = rf(q1.w);
        f.G.pitch = rf(q2.x), f.G.rp = rf(q2.y);
        f.job = f.band = 0;
        return f;
    };
    // issue(k): this wave's share of tile k's LDS-DMA into buffer k % 3 (nl = its load instructions), and
    // (all lanes) the tile's column / row tap tables
    const auto issue = [&](int k, int& nl) -> SplitTile {
        const int       buf = k % kSplitBufs;
        const SplitTile f   = get_geo(k);
        const int       sb  = L.stage + buf * L.stage_bytes;
        nl                  = 0;
        if (f.ok) {
            const JobS J = job_load(slot(k));
            stage_issue(J, f.G, sb, wave, nw);
            const int ni = (f.G.nr * f.G.ng + 63) >> 6; // DMA instructions i = wave, wave + nw, ...
            nl           = ni > wave ? (ni - wave + nw - 1) / nw : 0;
            const auto xt = lds_ptr<i32x2>(L.xt + buf * L.xt_bytes);
            for (int x = tid; x < W; x += nt) {
                const XTap c = xcoef<RESIZE_LINEAR>(JF(J, win_x) + x, JF(J, scale_x), JF(J, crop_w));
                xt[x]        = (i32x2){4 * (c.sx - f.G.u_lo), (c.a0 & 0xffff) | (c.a1 << 16)};
            }
            const auto yt = lds_ptr<i32x4>(L.yt + buf * kSplitTRMax * 16);
            for (int r = tid; r < f.nrows; r += nt) {
                const YTap y = ycoef<RESIZE_LINEAR>(JF(J, win_y) + f.y0 + r, JF(J, scale_y), JF(J, crop_h));
                yt[r]        = (i32x4){sb + (y.r0 - f.G.v_lo) * f.G.rp, sb + (y.r1 - f.G.v_lo) * f.G.rp, y.b0, y.b1};
            }
        }
        return f;
    };
    const auto unpack = [&](const SplitTile& f, int k) {
        if (f.ok) stage_unpack(job_load(slot(k)), f.G, L.stage + (k % kSplitBufs) * L.stage_bytes, wave, nw);
    };
    // compute(k): tile k from buffer k % 3; returns this wave's store instructions when the tile is a full
    // one (else -1: the caller's next counted wait drains)
    const auto compute = [&](int k) -> int {
        const int  buf  = k % kSplitBufs;
        const auto info = lds_ptr<const int32_t>(geo_slot(k));
        const bool ok   = __builtin_amdgcn_readfirstlane(info[0]) != 0;
        if (!ok) return 0;
        const int y0 = __builtin_amdgcn_readfirstlane(info[1]), nrows = __builtin_amdgcn_readfirstlane(info[2]);
        if (active) {
            const JobS   J = job_load(slot(k));
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
            i32x4 ytn = yt[min(lph, nrows - 1)]; // (the next row's taps read a row ahead)
            for (int ry = lph; ry < nrows; ry += nph) {
                const i32x4 ytr = ytn;
                if (ry + nph < nrows) ytn = yt[ry + nph];
                int         val[4][3];
                resize4_linear_scaled(ytr, col, wxk, val);
                if (TAIL && tmask) {
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        if (tmask & (1 << q)) {
                            const int x = flip ? W - 1 - (ox0 + q) : ox0 + q;
                            tail_fix<true>(ytr, col[q], wxk[q], (wx0 + x) * 3, xv, val[q]);
                        }
                }
                const int idx = (y0 + ry) * W + ox0;
                // the twelve LUT reads in flight together, then the three plane stores
                float lv[3][4];
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int q = 0; q < 4; q++) lv[c][q] = lut_at(c, val[q][c]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < 3; c++) {
                    const int oc = bgr ? 2 - c : c;
                    store_f32x4(orsrc, (oc * plane + idx) * 4, lv[c][0], lv[c][1], lv[c][2], lv[c][3]);
                }
            }
        }
        return nrows == TR ? s_full : -1;
    };

    // Prologue: the LUT (12 LDS-DMA instructions) and the first five tiles' jobs, one per wave; the first
    // three tiles' geometry; tiles 0 and 1 issued; tile 0 unpacked once its loads (not tile 1's) landed.
    for (int i = wave; i < 12 + min(K, 5); i += nw) {
        if (i < 12) lds_dma<4>(uniform_rsrc((const void*)a.lut, 3 * 256 * 4), L.lut + i * 256, (uint32_t)(lane * 4 + i * 256));
        else fetch_job(a, tile_of(i - 12), slot(i - 12));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (wave == nw - 1)
        for (int k = 0; k < min(K, 3); k++) put_geo(k);
    lds_barrier();
    int             nl0 = 0, nl1 = 0;
    const SplitTile f0 = issue(0, nl0);
    SplitTile       f1 = f0;
    f1.ok              = false;
    if (K > 1) f1 = issue(1, nl1);
    wait_vm_exact(nl1); // tile 0's loads
    unpack(f0, 0);
    lds_barrier(); // B0
    // Tile k: the job of tile k + 5 fetched (wave 0), tile k + 3's geometry (the last wave), tile k + 2
    // issued, tile k computed, then -- once this wave's loads of tile k + 1 landed: `after` counts the
    // operations it issued since them -- tile k + 1 unpacked; one barrier.  Jobs: a ring of six; a fetched
    // job is read three tiles later, after its fetcher's counted wait (the fetch precedes the next tile's
    // loads) and a barrier.
    int after = 0;
    for (int k = 0; k < K; k++) {
        stamp(k, 0), stamp(k, 8);
        int fj = 0;
        if (wave == 0 && k + 5 < K) fetch_job(a, tile_of(k + 5), slot(k + 5)), fj = 1;
        if (wave == nw - 1 && k + 3 < K) {
            // (uniform f64 work on one wave that shares its SIMD with compute waves: at raised priority, or
            // it gets issue slots only when they stall and the tile's barrier waits for it)
            __builtin_amdgcn_s_setprio(AEON_SPLIT_GEO_PRIO);
            put_geo(k + 3);
            __builtin_amdgcn_s_setprio(0);
        }
        int       nl2 = 0;
        SplitTile f2  = f1;
        f2.ok         = false;
        if (k + 2 < K) f2 = issue(k + 2, nl2);
        stamp(k, 1), stamp(k, 9);
        const int sk = compute(k);
        stamp(k, 2), stamp(k, 10);
        if (k + 1 < K) {
            wait_vm_exact(after < 0 || sk < 0 ? -1 : after + fj + nl2 + sk);
            stamp(k, 3), stamp(k, 11);
            unpack(f1, k + 1);
            stamp(k, 4), stamp(k, 12);
        }
        after = sk; // (the operations issued after tile k + 2's loads: tile k's stores)
        f1    = f2;
        lds_barrier(); // tile k computed (its buffer free), tile k + 1 unpacked
    }
#ifdef AEON_HIP_TRACE
    if (a.trace && tid == 0) a.trace[(blockIdx.x * 16 + 15) * 16 + 15] = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
}

hipError_t launch_split(bool tail, int occ, const LaunchArgs& a, const SplitArgs& s, int grid, hipStream_t stream,
                        hipEvent_t start, hipEvent_t stop)
{
    const void* fn      = occ == 2 ? (tail ? (const void*)augment_split<true, 2> : (const void*)augment_split<false, 2>)
                                   : (tail ? (const void*)augment_split<true, 1> : (const void*)augment_split<false, 1>);
    void*       args[2] = {(void*)&a, (void*)&s};
    if (start || stop) return hipExtLaunchKernel(fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream, start, stop, 0);
    return hipLaunchKernel(fn, dim3(grid), dim3(a.threads), args, a.lds_bytes, stream);
}

hipError_t split_lds_limit(int bytes)
{
    for (const void* fn : {(const void*)augment_split<true, 1>, (const void*)augment_split<false, 1>,
                           (const void*)augment_split<true, 2>, (const void*)augment_split<false, 2>}) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Workgroups of augment_split one CU holds at once for a launch shape.
hipError_t split_occupancy(bool tail, int occ, const LaunchArgs& a, int* blocks)
{
    const void* fn = occ == 2 ? (tail ? (const void*)augment_split<true, 2> : (const void*)augment_split<false, 2>)
                              : (tail ? (const void*)augment_split<true, 1> : (const void*)augment_split<false, 1>);
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, fn, a.threads, a.lds_bytes);
}

} // namespace aeon_hip
