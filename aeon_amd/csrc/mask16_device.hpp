// mask16_device.hpp -- device side of the single-channel NEAREST gather of pixel masks / depth maps:
// the LDS-staged row-block gather (row map, source-row copy, gather + stores) shared by the
// nearest_staged launch (mask16_kernels.hip) and the mask blocks the image tile kernel takes after
// its tiles in an image + mask call (augment_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aug_job.hpp"
#include "mask16.hpp"

namespace aeon_hip {

// Global (not flat) memory operations: a flat access also counts on the LDS counter, so waiting
// for an LDS read (say, the address a load needs) would wait for every flat load in flight too.
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(uint64_t a)
{
    return (__attribute__((address_space(1))) T*)a;
}

// 4 consecutive output elements of a row: one dword (uint8, saturated) or one 16-byte (float32)
// store when the destination is aligned, element stores otherwise
__device__ __forceinline__ void store4(const Mask16Job& J, size_t o, int nk, const uint32_t v[4])
{
    if (J.dtype != OUT_U8 && J.dtype != OUT_F32) { // the other convertTo targets, element by element
        for (int k = 0; k < nk; k++) {
            const uint32_t x = v[k];
            switch (J.dtype) {
            case OUT_S8: gptr<int8_t>(J.out_ptr)[o + k] = (int8_t)min(x, 127u); break;
            case OUT_S16: gptr<int16_t>(J.out_ptr)[o + k] = (int16_t)min(x, 32767u); break;
            case OUT_U16: gptr<uint16_t>(J.out_ptr)[o + k] = (uint16_t)x; break;
            case OUT_S32: gptr<int32_t>(J.out_ptr)[o + k] = (int32_t)x; break;
            default: gptr<double>(J.out_ptr)[o + k] = (double)x; break; // OUT_F64
            }
        }
        return;
    }
    if (J.dtype == OUT_F32) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        const uint64_t dst = J.out_ptr + o * 4;
        if (nk == 4 && (dst & 15) == 0) {
            const f32x4 q = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
            __builtin_nontemporal_store(q, gptr<f32x4>(dst));
        } else {
            for (int k = 0; k < nk; k++) gptr<float>(dst)[k] = (float)v[k];
        }
    } else {
        const uint64_t dst = J.out_ptr + o;
        const uint32_t b0 = min(v[0], 255u), b1 = min(v[1], 255u), b2 = min(v[2], 255u), b3 = min(v[3], 255u);
        if (nk == 4 && (dst & 3) == 0) {
            __builtin_nontemporal_store(b0 | (b1 << 8) | (b2 << 16) | (b3 << 24), gptr<uint32_t>(dst));
        } else {
            const uint32_t b[4] = {b0, b1, b2, b3};
            for (int k = 0; k < nk; k++) gptr<uint8_t>(dst)[k] = (uint8_t)b[k];
        }
    }
}

// LDS-staged gather (the default): a workgroup owns `rows` output rows of one record.  Wave 0 maps
// them to their source rows (sy = min(floor(y * ify), crop_h - 1), monotonic in y) and numbers the
// distinct ones; the workgroup copies each distinct row's crop segment into LDS with aligned
// 16-byte loads (a 16-byte-aligned block that holds one byte of the segment never leaves that
// byte's page, so the over-read at both ends is always mapped), and every lane then gathers its 16
// output columns from LDS and stores them as one 16-byte row piece.  Compared with the direct
// gather above, the texture path sees one 16-byte load per 16 source bytes instead of one byte load
// per output element, and one 16-byte store per 16 output bytes.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kLoadsPerLane = 8; // 16-byte loads a lane keeps in flight before their LDS writes

// The source rows of one block of output rows, as wave 0 numbered them.
// Kept small (336 B of static LDS): with the staged rows sized to the distinct rows a block can
// touch, C5's 512-row masks fit four workgroups per CU, i.e. their 1,024 blocks in one round.
struct RowMap {
    uint32_t off[64];  // byte offset from src_ptr of each distinct row's crop segment
    uint8_t  slot[64]; // output row -> distinct row
    int      nslots, nrows, rec, y0;
};
__device__ __forceinline__ uint64_t seg_start(const Mask16Job& J, const RowMap& M, int s) { return J.src_ptr + M.off[s]; }

// wave 0: rows [y0, y0 + nrows) of record `rec`
// (max_slots: the staged rows the launch's LDS holds -- the host's exact bound on the distinct
// rows of any block, so the clamp never applies)
__device__ __forceinline__ void map_rows(const Mask16Job& J, int rec, int y0, int nrows, int max_slots, RowMap& M)
{
    const int  tid   = threadIdx.x;
    const int  eb    = J.src_elem;
    const bool valid = tid < nrows;
    const int  sy    = valid ? min((int)floor((y0 + tid) * J.scale_y), J.crop_h - 1) : -1;
    const int  prev  = __shfl_up(sy, 1);
    const bool fresh = valid && (tid == 0 || sy != prev);
    const unsigned long long m    = __ballot(fresh);
    const unsigned long long upto = tid == 63 ? ~0ull : ((2ull << tid) - 1);
    const int                slot = __popcll(m & upto) - 1;
    if (valid) M.slot[tid] = (uint8_t)slot;
    if (fresh) M.off[slot] = (uint32_t)((uint64_t)(J.crop_y + sy) * J.src_stride + (uint64_t)J.crop_x * eb);
    if (tid == 0) M.nslots = min(__popcll(m), max_slots), M.nrows = nrows, M.rec = rec, M.y0 = y0;
}

__device__ __forceinline__ int seg_blocks(const Mask16Job& J) { return (15 + J.crop_w * J.src_elem + 15) >> 4; }

// Source-row copy: thread t moves 16-byte blocks t, t + blockDim, ... of the concatenated row
// segments (block i = row i / nblk, block i % nblk, the quotient through a float reciprocal: exact
// while i / nblk < 2^12 as (i + 0.5) / nblk stays > 0.5 / nblk from an integer).  Each thread
// issues kLoadsPerLane loads before their LDS writes; the loads are unconditional (clamped to the
// last block) because a branch around each would make the compiler wait for it at the join.
template <int LPL = kLoadsPerLane>
__device__ __forceinline__ void copy_rows(const Mask16Job& J, const RowMap& M, int nblk, int pitch, uint8_t* lds)
{
    constexpr int kLoadsPerLane = LPL;
    const int   total = M.nslots * nblk;
    const float rcp   = 1.0f / (float)nblk;
    if (total <= 0) return;
    for (int i0 = threadIdx.x; i0 < total; i0 += kLoadsPerLane * blockDim.x) {
        u32x4 v[kLoadsPerLane];
        int   at[kLoadsPerLane];
#pragma unroll
        for (int u = 0; u < kLoadsPerLane; u++) {
            const int i = min(i0 + u * (int)blockDim.x, total - 1);
            const int s = (int)(((float)i + 0.5f) * rcp), b = i - s * nblk;
            v[u]        = __builtin_nontemporal_load(gptr<const u32x4>((seg_start(J, M, s) & ~(uint64_t)15) + (uint64_t)b * 16));
            at[u]       = s * pitch + b * 16;
        }
#pragma unroll
        for (int u = 0; u < kLoadsPerLane; u++)
            if (i0 + u * (int)blockDim.x < total) *(u32x4*)(lds + at[u]) = v[u];
    }
}

// 8-bit source, 8-bit output, and every 4 consecutive output columns of the lane drawn from 5
// consecutive source bytes (horizontal scale < 4/3): per 4 outputs, one 8-byte LDS read pair and one
// v_perm_b32 (selector = the 4 source bytes' positions in the pair) instead of 4 byte reads, 4
// saturations and the packing.  Returns false when a lane's columns do not qualify.
__device__ __forceinline__ bool gather_u8_perm(const Mask16Job& J, const RowMap& M, int pitch, const uint8_t* lds,
                                               int x0, int r0, int rstep, const int (&sx)[16])
{
    int      lo[4];
    uint32_t rel[4];
    bool     ok = true;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const int a = sx[4 * w], d = sx[4 * w + 3]; // ascending, or descending when flipped
        lo[w]       = min(a, d);
        ok          = ok && (max(a, d) - lo[w] <= 4);
        rel[w]      = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) rel[w] |= (uint32_t)(sx[4 * w + k] - lo[w]) << (8 * k);
    }
    if (!ok) return false;
    const uint32_t* lds32 = (const uint32_t*)lds;
    for (int r = r0; r < M.nrows; r += rstep) {
        const int s    = M.slot[r];
        const int rowb = s * pitch + (int)(seg_start(J, M, s) & 15);
        u32x4     q;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const int      a   = rowb + lo[w];
            const uint32_t sel = rel[w] + (uint32_t)(a & 3) * 0x01010101u;
            q[w]               = __builtin_amdgcn_perm(lds32[(a >> 2) + 1], lds32[a >> 2], sel);
        }
        __builtin_nontemporal_store(q, gptr<u32x4>(J.out_ptr + (size_t)(M.y0 + r) * J.out_pitch + x0));
    }
    return true;
}

template <typename T>
__device__ __forceinline__ void gather_rows(const Mask16Job& J, const RowMap& M, int pitch, const uint8_t* lds,
                                            bool perm_ok)
{
    constexpr int eb    = sizeof(T);
    constexpr int C     = 16; // output columns per lane
    const int     tid   = threadIdx.x;
    const int     nrows = M.nrows, y0 = M.y0;
    const int     ng    = (J.out_w + C - 1) / C;
    const int     per   = min(ng, (int)blockDim.x);
    const int     rstep = blockDim.x / per;
    const int     r0    = tid / per;
    if (r0 >= rstep) return;
    const bool u8out = J.dtype == OUT_U8;
    for (int g = tid % per; g < ng; g += per) {
        const int x0 = g * C;
        const int nk = min(C, J.out_w - x0);
        int       off[C];
#pragma unroll
        for (int k = 0; k < C; k++) {
            const int x  = min(x0 + k, J.out_w - 1);
            const int dx = J.flip ? J.out_w - 1 - x : x; // cv::flip(.., 1) after the resize
            off[k]       = min((int)floor(dx * J.scale_x), J.crop_w - 1) * eb;
        }
        if (eb == 1 && u8out && nk == C && perm_ok && ((J.out_ptr + (size_t)y0 * J.out_pitch + x0) & 15) == 0 &&
            (J.out_pitch & 15) == 0 && gather_u8_perm(J, M, pitch, lds, x0, r0, rstep, off))
            continue;
        for (int r = r0; r < nrows; r += rstep) {
            const int      s    = M.slot[r];
            const uint8_t* base = lds + s * pitch + (int)(seg_start(J, M, s) & 15);
            uint32_t       v[C];
#pragma unroll
            for (int k = 0; k < C; k++) v[k] = *(const T*)(base + off[k]);
            const size_t o = (size_t)(y0 + r) * J.out_pitch + x0;
            if (u8out) {
                const uint64_t dst = J.out_ptr + o;
                if (nk == C && (dst & 15) == 0) {
                    u32x4 q;
#pragma unroll
                    for (int w = 0; w < 4; w++)
                        q[w] = min(v[4 * w], 255u) | (min(v[4 * w + 1], 255u) << 8) | (min(v[4 * w + 2], 255u) << 16) |
                               (min(v[4 * w + 3], 255u) << 24);
                    __builtin_nontemporal_store(q, gptr<u32x4>(dst));
                    continue;
                }
            }
#pragma unroll
            for (int w = 0; w < 4; w++)
                if (4 * w < nk) store4(J, o + 4 * w, min(4, nk - 4 * w), v + 4 * w);
        }
    }
}

__device__ __forceinline__ void gather_any(const Mask16Job& J, const RowMap& M, int pitch, const uint8_t* lds,
                                           bool perm_ok)
{
    if (J.src_elem == 2) gather_rows<uint16_t>(J, M, pitch, lds, false);
    else gather_rows<uint8_t>(J, M, pitch, lds, perm_ok);
}

} // namespace aeon_hip
