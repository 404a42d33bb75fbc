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

// An image + mask launch (augment_kernels.hip mask_blocks): LDS bytes ahead of a row block's staged
// rows -- the row map (336 B, 16-aligned), the block's job (80 B) and the draw word (16 B).
constexpr int kMaskBlockHdrBytes = 336 + 80 + 16;

// LDS-staged gather (nearest_staged) geometry, shared by the host and the launch: bytes per
// staged source row (a 16-byte-aligned window around the crop segment) and output rows per
// workgroup (up to 64 rows / ~32K output elements per workgroup, LDS <= 64 KB).
inline int mask16_pitch(int max_seg_bytes) { return (max_seg_bytes + 15 + 15) & ~15; }
inline int mask16_rows(int max_w, int max_seg_bytes)
{
    const int pitch = mask16_pitch(max_seg_bytes);
    int       r     = 64 < 65536 / pitch ? 64 : 65536 / pitch;
    const int by_w  = 32768 / (max_w > 1 ? max_w : 1);
    return r < (by_w > 1 ? by_w : 1) ? r : (by_w > 1 ? by_w : 1);
}

} // namespace aeon_hip
