// mask16_kernels.hip -- the single-channel NEAREST gather pass of the pixel-mask / depth-map path
// for rotation-free records: 8-bit (CV_8U) and 16-bit (CV_16U) sources.  aeon decodes both with
// CV_LOAD_IMAGE_ANYDEPTH (src/etl_pixel_mask.cpp:30-53, src/etl_depthmap.cpp:30-53), so a 16-bit
// PNG stays 16-bit, and the transformer is crop -> cv::resize INTER_NEAREST -> cv::flip
// (etl_pixel_mask.cpp:65-92, etl_depthmap.cpp:65-96); the loader then converts to the output
// type (image::convert_mix_channels -> convertTo, src/image.cpp:176-212): saturate_cast<uchar>
// for uint8 output, exact for float.
//
// NEAREST is a pure gather, so this is one pass with no LDS staging: every output pixel reads
// one source element (the source rows a workgroup touches stay in L1/L2).  A workgroup owns
// `rows` output rows of one record; a lane owns 4 consecutive output columns of those rows, so
// their source columns x_ofs = min(floor(dx * ifx), sw - 1) (ifx in double, OpenCV's resizeNN;
// flip folded into dx) are computed once, and the 4 results leave as one dword (uint8) or one
// 16-byte (float32) store when the destination is aligned.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "aug_job.hpp"
#include "mask16.hpp"
#include "mask16_device.hpp"

namespace aeon_hip {

template <typename T>
__device__ __forceinline__ void nearest_rows(const Mask16Job& J, int y0, int y1)
{
    const uint8_t* src = (const uint8_t*)J.src_ptr;
    const int      ng  = (J.out_w + 3) >> 2;
    for (int g = threadIdx.x; g < ng; g += blockDim.x) {
        const int x0 = g * 4;
        const int nk = min(4, J.out_w - x0);
        int       sx[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int x  = min(x0 + k, J.out_w - 1);
            const int dx = J.flip ? J.out_w - 1 - x : x; // cv::flip(.., 1) after the resize
            sx[k]        = min((int)floor(dx * J.scale_x), J.crop_w - 1);
        }
        // rows in chunks of 8: every gather of the chunk is issued before its stores (the
        // compiler may not hoist loads over stores through these untyped pointers itself)
        for (int yc = y0; yc < y1; yc += 8) {
            uint32_t v[8][4];
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int y   = min(yc + r, y1 - 1);
                const int sy  = min((int)floor(y * J.scale_y), J.crop_h - 1);
                const auto row = gptr<const T>((uint64_t)(src + (size_t)(J.crop_y + sy) * J.src_stride)) + J.crop_x;
#pragma unroll
                for (int k = 0; k < 4; k++) v[r][k] = row[sx[k]];
            }
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const int y = yc + r;
                if (y >= y1) break;
                store4(J, (size_t)y * J.out_pitch + x0, nk, v[r]);
            }
        }
    }
}

// The workgroup's job, loaded once.  The table may be the caller's pinned ring slot, which the host
// rewrote since the GPU last read that memory: the first lanes read it dword by dword at system scope
// (sc0 sc1, through to the host, like the tile kernel's fetch_job) into LDS, and every lane copies it.
__device__ __forceinline__ Mask16Job load_job(const Mask16Job* src, Mask16Job& lds)
{
    constexpr int kWords = (int)(sizeof(Mask16Job) / 4);
    static_assert(sizeof(Mask16Job) % 4 == 0 && kWords <= 64, "Mask16Job: whole dwords, one wave");
    if (threadIdx.x < kWords)
        reinterpret_cast<uint32_t*>(&lds)[threadIdx.x] = __hip_atomic_load(
            reinterpret_cast<const uint32_t*>(src) + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    return lds;
}

// one block of rows per workgroup: grid (row blocks, records)
__global__ __launch_bounds__(256) void nearest_staged(const Mask16Job* __restrict__ jobs, int rows_per_block, int pitch,
                                                      int perm_ok, int max_slots)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_rows[];
    __shared__ RowMap M;
    __shared__ Mask16Job Js;
    const Mask16Job J = load_job(jobs + blockIdx.y, Js);
    const int        y0 = blockIdx.x * rows_per_block;
    if (y0 >= J.out_h) return;
    if (threadIdx.x < 64) map_rows(J, blockIdx.y, y0, min(rows_per_block, J.out_h - y0), max_slots, M);
    __syncthreads();
    copy_rows(J, M, seg_blocks(J), pitch, lds_rows);
    __syncthreads();
    gather_any(J, M, pitch, lds_rows, perm_ok != 0);
}

__global__ __launch_bounds__(256) void nearest_records(const Mask16Job* __restrict__ jobs, int rows_per_block)
{
    __shared__ Mask16Job Js;
    const Mask16Job J = load_job(jobs + blockIdx.y, Js);
    const int        y0 = blockIdx.x * rows_per_block;
    if (y0 >= J.out_h) return;
    const int y1 = min(y0 + rows_per_block, J.out_h);
    if (J.src_elem == 2) nearest_rows<uint16_t>(J, y0, y1);
    else nearest_rows<uint8_t>(J, y0, y1);
}

hipError_t launch_nearest(const Mask16Job* jobs, int n_jobs, int max_h, int max_w, int max_seg_bytes, int max_slots,
                          hipStream_t stream, hipEvent_t start, hipEvent_t stop)
{
    if (n_jobs <= 0) return hipSuccess;
    const int pitch = mask16_pitch(max_seg_bytes);
    // staged: up to 64 output rows / ~32K output elements per workgroup, LDS <= 64 KB (C5 A/B:
    // 64 rows 15.8 us, 32 rows 16.7, 16 rows 20.5, 8 rows 29.9; the direct gather 26.3); the LDS
    // holds max_slots staged rows (the host's bound on the distinct source rows of one block).
    // Rows longer than the staging holds (srows < 1) take the direct gather.
    const int srows = mask16_rows(max_w, max_seg_bytes);
    if (srows >= 1) {
        max_slots       = std::max(1, std::min(max_slots, srows));
        const dim3 grid((max_h + srows - 1) / srows, n_jobs);
        const size_t lds = (size_t)max_slots * pitch;
        int perm = 1; // gather_u8_perm where the columns qualify
        if (start || stop) {
            void* args[5] = {(void*)&jobs, (void*)&srows, (void*)&pitch, (void*)&perm, (void*)&max_slots};
            return hipExtLaunchKernel((const void*)nearest_staged, grid, dim3(256), args, lds, stream, start, stop, 0);
        }
        hipLaunchKernelGGL(nearest_staged, grid, dim3(256), lds, stream, jobs, srows, pitch, perm, max_slots);
        return hipGetLastError();
    }
    // lanes = the widest record's 4-column groups (64..256); ~8K output pixels per workgroup
    const int groups  = (max_w + 3) / 4;
    const int threads = std::min(256, std::max(64, (groups + 63) / 64 * 64));
    int       rows    = std::max(1, std::min(64, 8192 / std::max(1, max_w)));
    const dim3 grid((max_h + rows - 1) / rows, n_jobs);
    if (start || stop) { // dispatch-stamped timing events, as the tile kernels
        void* args[2] = {(void*)&jobs, (void*)&rows};
        return hipExtLaunchKernel((const void*)nearest_records, grid, dim3(threads), args, 0, stream, start, stop, 0);
    }
    hipLaunchKernelGGL(nearest_records, grid, dim3(threads), 0, stream, jobs, rows);
    return hipGetLastError();
}

} // namespace aeon_hip
