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
class thread_pool;
// shared: entropy-decode on that pool (the decoder's own, pinned to its cpu_list -- aeon's extract
// runs inside provide() on the decode pool); null: a pool of the stage's own (thread_affinity_map)
JpegState* jpeg_state_create(thread_pool* shared = nullptr);
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
    int32_t  up[3];     // JpegUpsample of each component (host-chosen: no divisions per pixel)
    int32_t  hf[3], vf[3]; // hmax / hs, vmax / vs
    int32_t  pad2_;
    uint16_t q[3][64];  // quantisation table of each component, natural order
};

// jdsample.c's upsampler of a component, chosen per file on the host.
enum JpegUpsample : int32_t {
    UP_FULL = 0, // full resolution
    UP_H2V1 = 1, // h2v1_fancy_upsample
    UP_H1V2 = 2, // h1v2_fancy_upsample (libjpeg-turbo)
    UP_H2V2 = 3, // h2v2_fancy_upsample
    UP_BOX  = 4, // h2v1 / h2v2 / int_upsample box replication (other ratios, components < 3 samples wide)
};

// IDCT work item: blocks [first, first + count) of component `comp` of image `img`.
struct JpegChunk {
    int32_t img, comp, first, count;
};

// Colour work item: output rows [y0, y0 + rows) of image `img`.
struct JpegRows {
    int32_t img, y0, rows, pad_;
};

constexpr int kJpegIdctLanes  = 256;                             // IDCT workgroup: 8 lanes per block
constexpr int kJpegIdctUnroll = 4;                               // blocks per lane group
constexpr int kJpegIdctBlocks = kJpegIdctLanes / 8 * kJpegIdctUnroll; // blocks per IDCT workgroup (chunk)
constexpr int kJpegRowsPerWg = 8;   // output rows per colour workgroup (fewer when the staged rows outgrow LDS)
constexpr int kJpegColorLds  = 160 * 1024; // most LDS a colour workgroup stages

// jdsample.c's choice for a component (h / v expansion factors, dw samples per row): fancy
// upsampling needs 3+ samples per row.
inline int jpeg_upsample_mode(int hf, int vf, int dw)
{
    const bool fancy = dw > 2;
    if (hf == 1 && vf == 1) return UP_FULL;
    if (hf == 2 && vf == 1 && fancy) return UP_H2V1;
    if (hf == 1 && vf == 2 && fancy) return UP_H1V2;
    if (hf == 2 && vf == 2 && fancy) return UP_H2V2;
    return UP_BOX;
}

// Plane rows the colour pass stages for a band of `rows` output rows of a component (a bound; the
// kernel stages the exact range).
inline int jpeg_stage_rows(int up, int vf, int rows)
{
    if (up == UP_H1V2 || up == UP_H2V2) return rows / 2 + 3;
    if (up == UP_BOX) return rows / vf + 2;
    return rows;
}

} // namespace aeon_hip
