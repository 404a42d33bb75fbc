// jpeg.hpp -- the JPEG decode stage of image::extractor::extract (aeon src/etl_image.cpp:83-99):
// descriptors shared by the host entropy decoder (jpeg_host.cpp) and the GPU kernels
// (jpeg_kernels.hip).
//
// Split: Huffman decoding is a serial bit-stream walk per file, so it runs on the host pool (one
// file per task); everything per pixel -- dequantisation, the ISLOW IDCT, fancy upsampling and the
// YCbCr -> BGR conversion -- runs on the GPU, which writes the decoded HWC records straight into the
// device source arena the augmentation kernels read.  What crosses PCIe is the sparse coefficient
// stream: per 8x8 block a 64-bit zigzag mask of its non-zero coefficients plus those values (int16),
// typically a fraction of the decoded pixels' bytes.
#pragma once
#include <stdint.h>

#include <stdexcept>
#include <string>

namespace aeon_hip {

// Host-side error of the JPEG stage, carrying its AEON_HIP_E* code across to the C ABI.
struct jpeg_error : std::runtime_error {
    int code;
    jpeg_error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct JpegState;
JpegState* jpeg_state_create();
void       jpeg_state_destroy(JpegState* s);

// One 8x8 block: bit z of `mask` = zigzag coefficient z is non-zero; its values follow in zigzag
// order at values[val_off ...] of the block's image.
struct alignas(16) JpegBlock {
    uint64_t mask;
    uint32_t val_off;
    uint32_t pad_;
};

// One file of a decode call, as the kernels see it (device addresses).
struct alignas(16) JpegImage {
    uint64_t blocks[3]; // JpegBlock[bh][bw] per component
    uint64_t values;    // int16 coefficient values
    uint64_t planes[3]; // IDCT output per component: (bw*8) x (bh*8) uint8, row pitch bw*8
    uint64_t out;       // decoded record: HWC uint8 (BGR or gray), out_stride bytes per row
    int32_t  W, H, ncomp, out_cn, out_stride, hmax, vmax, pad_;
    int32_t  bw[3], bh[3], dw[3], dh[3], hs[3], vs[3];
    uint16_t q[3][64];  // quantisation table of each component, natural order
};

// IDCT work item: blocks [first, first + count) of component `comp` of image `img`.
struct JpegChunk {
    int32_t img, comp, first, count;
};

// Colour work item: output rows [y0, y0 + rows) of image `img`.
struct JpegRows {
    int32_t img, y0, rows, pad_;
};

constexpr int kJpegIdctLanes = 128; // blocks per IDCT workgroup (one lane per block)
constexpr int kJpegRowsPerWg = 4;   // output rows per colour workgroup

} // namespace aeon_hip
