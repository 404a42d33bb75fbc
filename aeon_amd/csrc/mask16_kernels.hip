// mask16_kernels.hip -- 16-bit (CV_16U) single-channel records of the pixel-mask / depth-map
// path: aeon decodes both with CV_LOAD_IMAGE_ANYDEPTH (src/etl_pixel_mask.cpp:30-53,
// src/etl_depthmap.cpp:30-53), so a 16-bit PNG stays 16-bit, and the transformer is
// crop -> cv::resize INTER_NEAREST -> cv::flip (etl_pixel_mask.cpp:65-92, etl_depthmap.cpp:65-96);
// the loader then converts to the output type (image::convert_mix_channels -> convertTo,
// src/image.cpp:176-212): saturate_cast<uchar> for uint8 output, exact for float.
//
// NEAREST is a pure gather, so this is one pass: every output pixel reads one source element.
// A workgroup owns output rows of one record (256 lanes across the row); the column index is
// OpenCV's resizeNN x_ofs = min(floor(dx * ifx), sw - 1) with ifx in double, as the 8-bit path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mask16.hpp"

namespace aeon_hip {

__global__ __launch_bounds__(256) void nearest16_records(const Mask16Job* __restrict__ jobs, int rows_per_block)
{
    const Mask16Job& J = jobs[blockIdx.y];
    const int        y0 = blockIdx.x * rows_per_block;
    if (y0 >= J.out_h) return;
    const uint8_t* src = (const uint8_t*)J.src_ptr;
    const int      y1  = min(y0 + rows_per_block, J.out_h);
    for (int y = y0; y < y1; y++) {
        const int      sy  = min((int)floor(y * J.scale_y), J.crop_h - 1);
        const uint16_t* row = (const uint16_t*)(src + (size_t)(J.crop_y + sy) * J.src_stride) + J.crop_x;
        for (int x = threadIdx.x; x < J.out_w; x += blockDim.x) {
            const int dx = J.flip ? J.out_w - 1 - x : x; // cv::flip(.., 1) after the resize
            const int sx = min((int)floor(dx * J.scale_x), J.crop_w - 1);
            const uint32_t v  = row[sx];
            const size_t   o  = (size_t)y * J.out_pitch + x;
            if (J.dtype == 1) ((float*)J.out_ptr)[o] = (float)v;
            else ((uint8_t*)J.out_ptr)[o] = (uint8_t)min(v, 255u);
        }
    }
}

hipError_t launch_nearest16(const Mask16Job* jobs, int n_jobs, int max_h, hipStream_t stream)
{
    if (n_jobs <= 0) return hipSuccess;
    constexpr int rows = 4;
    hipLaunchKernelGGL(nearest16_records, dim3((max_h + rows - 1) / rows, n_jobs), dim3(256), 0, stream, jobs,
                       rows);
    return hipGetLastError();
}

} // namespace aeon_hip
