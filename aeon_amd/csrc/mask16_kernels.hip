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

#include "aug_job.hpp"
#include "mask16.hpp"

namespace aeon_hip {

// 4 consecutive output elements of a row: one dword (uint8, saturated) or one 16-byte (float32)
// store when the destination is aligned, element stores otherwise
__device__ __forceinline__ void store4(const Mask16Job& J, size_t o, int nk, const uint32_t v[4])
{
    if (J.dtype != OUT_U8 && J.dtype != OUT_F32) { // the other convertTo targets, element by element
        for (int k = 0; k < nk; k++) {
            const uint32_t x = v[k];
            switch (J.dtype) {
            case OUT_S8: ((int8_t*)J.out_ptr)[o + k] = (int8_t)min(x, 127u); break;
            case OUT_S16: ((int16_t*)J.out_ptr)[o + k] = (int16_t)min(x, 32767u); break;
            case OUT_U16: ((uint16_t*)J.out_ptr)[o + k] = (uint16_t)x; break;
            case OUT_S32: ((int32_t*)J.out_ptr)[o + k] = (int32_t)x; break;
            default: ((double*)J.out_ptr)[o + k] = (double)x; break; // OUT_F64
            }
        }
        return;
    }
    if (J.dtype == OUT_F32) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        float* dst = (float*)J.out_ptr + o;
        if (nk == 4 && ((uintptr_t)dst & 15) == 0) {
            const f32x4 q = {(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
            __builtin_nontemporal_store(q, (f32x4*)dst);
        } else {
            for (int k = 0; k < nk; k++) dst[k] = (float)v[k];
        }
    } else {
        uint8_t*       dst = (uint8_t*)J.out_ptr + o;
        const uint32_t b0 = min(v[0], 255u), b1 = min(v[1], 255u), b2 = min(v[2], 255u), b3 = min(v[3], 255u);
        if (nk == 4 && ((uintptr_t)dst & 3) == 0) {
            __builtin_nontemporal_store(b0 | (b1 << 8) | (b2 << 16) | (b3 << 24), (uint32_t*)dst);
        } else {
            const uint32_t b[4] = {b0, b1, b2, b3};
            for (int k = 0; k < nk; k++) dst[k] = (uint8_t)b[k];
        }
    }
}

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
                const T*  row = (const T*)(src + (size_t)(J.crop_y + sy) * J.src_stride) + J.crop_x;
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

__global__ __launch_bounds__(256) void nearest_records(const Mask16Job* __restrict__ jobs, int rows_per_block)
{
    const Mask16Job& J  = jobs[blockIdx.y];
    const int        y0 = blockIdx.x * rows_per_block;
    if (y0 >= J.out_h) return;
    const int y1 = min(y0 + rows_per_block, J.out_h);
    if (J.src_elem == 2) nearest_rows<uint16_t>(J, y0, y1);
    else nearest_rows<uint8_t>(J, y0, y1);
}

hipError_t launch_nearest(const Mask16Job* jobs, int n_jobs, int max_h, int max_w, hipStream_t stream,
                          hipEvent_t start, hipEvent_t stop)
{
    if (n_jobs <= 0) return hipSuccess;
    // lanes = the widest record's 4-column groups (64..256); ~8K output pixels per workgroup
    const int groups  = (max_w + 3) / 4;
    const int threads = std::min(256, std::max(64, (groups + 63) / 64 * 64));
    int       rows    = std::max(1, std::min(64, 8192 / std::max(1, max_w)));
    if (const char* e = std::getenv("AEON_HIP_NEAREST_ROWS")) rows = std::max(1, std::atoi(e)); // experiments
    const dim3 grid((max_h + rows - 1) / rows, n_jobs);
    if (start || stop) { // dispatch-stamped timing events, as the tile kernels
        void* args[2] = {(void*)&jobs, (void*)&rows};
        return hipExtLaunchKernel((const void*)nearest_records, grid, dim3(threads), args, 0, stream, start, stop, 0);
    }
    hipLaunchKernelGGL(nearest_records, grid, dim3(threads), 0, stream, jobs, rows);
    return hipGetLastError();
}

} // namespace aeon_hip
