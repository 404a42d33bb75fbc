// mask16.hpp -- job descriptor of the single-channel NEAREST pass of pixel masks / depth maps
// (mask16_kernels.hip): 16-bit sources, and rotation-free 8-bit ones.
#pragma once
#include <stdint.h>

namespace aeon_hip {

// One single-channel record: crop -> INTER_NEAREST resize -> flip -> convert.
struct alignas(16) Mask16Job {
    double   scale_x, scale_y;        // OpenCV's ifx/ify = 1 / (dst / src), as the 8-bit path
    uint64_t src_ptr;                 // device address of the (rotation-free) record
    uint64_t out_ptr;                 // output item
    int32_t  src_stride;              // bytes per source row
    int32_t  crop_x, crop_y, crop_w, crop_h;
    int32_t  out_w, out_h, out_pitch; // output size; elements per output row (canvas width
                                      // with fixed_aspect_ratio)
    int32_t  flip;
    int32_t  dtype;                   // OutDtype (AEON_DTYPE_*): saturating convertTo
    int32_t  src_elem;                // bytes per source element: 1 (CV_8U) or 2 (CV_16U)
    int32_t  src_scratch;             // host bookkeeping: src_ptr is an offset in the slot scratch
                                      // (the record's image::rotate pre-pass output)
};

} // namespace aeon_hip
