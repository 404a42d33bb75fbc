// jpeg.hpp -- the JPEG decode stage of image::extractor::extract (aeon src/etl_image.cpp:83-99):
// descriptors shared by the host entropy decoder (jpeg_host.cpp) and the GPU kernels
// (jpeg_kernels.hip).
//
// Split: the host pool parses each file's markers and tables.  A sequential file whose one scan
// carries every component (baseline / extended, interleaved, or a grayscale scan) then goes to the GPU
// whole: the host only unstuffs its entropy-coded bytes (splitting them at RSTn markers) into the
// staging buffer, and jpeg_huff (jpeg_huff.hip) Huffman-decodes them -- subsequences of
// a few hundred bits decoded in parallel, self-synchronising from guessed starts, then a prefix sum
// of block counts and DC differences and a final decode that writes every block's coefficients.
// Progressive and multi-scan files are entropy-decoded on the host pool into the sparse stream (per
// 8x8 block a 64-bit zigzag mask of its non-zero coefficients plus those values, int16).  Everything
// per pixel -- dequantisation, the ISLOW IDCT, fancy upsampling and the YCbCr -> BGR conversion --
// runs on the GPU, which writes the decoded HWC records straight into the device source arena the
// augmentation kernels read.
#pragma once
#include <stddef.h>
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
// runs inside provide() on the decode pool); null: a pool of the stage's own (thread_affinity_map).
// gpu_huff false: every file through the host entropy decoder (AEON_HIP_JPEG_HUFF=host, A/B runs)
JpegState* jpeg_state_create(thread_pool* shared = nullptr, bool gpu_huff = true);
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
    uint64_t values;    // int16 coefficient values (sparse stream: host-decoded files)
    uint64_t dvals[3];  // GPU-decoded files: 64 int16 per block (zigzag order, the mask's bits valid), else 0
    uint64_t planes[3]; // IDCT output per component: (bw*8) x (bh*8) uint8, row pitch bw*8
    uint64_t out;       // decoded record: HWC uint8 (BGR or gray), out_stride bytes per row
    int32_t  W, H, ncomp, out_cn, out_stride, hmax, vmax, pad_;
    int32_t  bw[3], bh[3], dw[3], dh[3], hs[3], vs[3];
    int32_t  up[3];     // JpegUpsample of each component (host-chosen: no divisions per pixel)
    int32_t  hf[3], vf[3]; // hmax / hs, vmax / vs
    int32_t  pad2_;
    uint16_t q[3][64];  // quantisation table of each component, natural order
    uint16_t pad3_[4];
    uint16_t qz[3][64]; // the same in zigzag order (the dense path of jpeg_idct: 16-byte loads)
};
static_assert(offsetof(JpegImage, qz) % 16 == 0, "JpegImage.qz: 16-byte rows");

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

// ---- GPU entropy decoding (jpeg_huff.hip) ----

constexpr int kHuffSubMin   = 256;  // subsequence (the bits one lane decodes per pass): per file, the
constexpr int kHuffSubMax   = 2048; // multiple of 32 in [min, max] nearest to spreading it over the lanes
constexpr int kHuffLanes    = 512;  // jpeg_huff workgroup (one per file, two per CU; AEON_HIP_JPEG_HUFF_LANES=1024 / 256)
constexpr int kHuffMaxBpm   = 10;   // blocks per MCU (libjpeg's D_MAX_BLOCKS_IN_MCU; the parser refuses more)
constexpr int kHuffFastBits = 10;   // lookahead of the LDS decode tables
constexpr int kHuffLeadBits = 512;  // a guessed walk starts this far before its subsequence (re-synchronising)
#ifndef AEON_HUFF_PROBE
constexpr int kHuffStageMax = 84 * 1024; // a file's data up to this is copied into LDS for its walks
#else
constexpr int kHuffStageMax = 80 * 1024; // (probe builds hold their stamps in LDS too)
#endif

// One DHT table as the file defines it (code lengths 1..16, then the symbols), validated on the host.
constexpr int kJpegHuffSlots = 4; // Huffman tables a GPU-decoded scan holds: two DC, two AC
struct JpegHuffTab {
    uint8_t counts[16];
    uint8_t symbols[256];
};

// A restart interval of a scan (the whole scan without DRI): its unstuffed bytes, as bit offsets into
// the file's data; its subsequences are [first_sub, first_sub + nsub) of the file.
struct JpegHuffSeg {
    uint32_t start_bit, end_bit;
    int32_t  first_sub, nsub;
};

// Per-subsequence device scratch: start / end decoder state (bit position | block-in-MCU << 32 |
// zigzag index << 40), blocks started and DC differences per component, their exclusive sums.
struct alignas(16) JpegHuffSub {
    uint64_t st, en;
    int32_t  cnt[4]; // blocks started, DC difference sums of components 0..2
    int32_t  ex[4];  // exclusive prefix of cnt over the file's subsequences
};

// One GPU-decoded file (device addresses).
struct alignas(16) JpegHuffFile {
    uint64_t data;      // unstuffed entropy-coded bytes, 4-byte aligned, segments back to back
    uint64_t segs;      // JpegHuffSeg[nseg]
    uint64_t sub_seg;   // int32 per subsequence: its segment
    uint64_t tabs;      // JpegHuffTab[kJpegHuffSlots]: the scan's DC tables in slots 0-1, AC in 2-3
    uint64_t subs;      // JpegHuffSub[nsub] (device scratch)
    uint64_t blocks[3]; // JpegBlock[bh][bw] per frame component (zeroed before the launch)
    uint64_t dvals[3];  // 64 int16 per block per frame component
    uint64_t blk_tab[2]; // byte c (c < kHuffMaxBpm) = MCU block c: frame component | x << 2 | y << 4 |
                         // its DC table slot << 6 | (its AC table slot - 2) << 7
    int32_t  nseg, nsub, restart, n_mcu; // restart: MCUs per segment (n_mcu without DRI)
    int32_t  bpm, mcux, ncomp;           // a non-interleaved (grayscale) scan: bpm 1, mcux = blocks per row
    int32_t  truncated; // first segment whose data ends with the file, not a marker (reading past it is an error); -1: none
    int32_t  bw[3], hs[3], vs[3], sub_bits; // sub_bits: the file's subsequence length
    int32_t  data_words, pad_[3];           // the data's 32-bit words (padding included)
};

// Device error word bit of a GPU-decoded file whose entropy-coded data is corrupt or truncated.
constexpr int kJpegCorruptBit = 256;

constexpr int kJpegIdctLanes  = 256;                             // IDCT workgroup: 8 lanes per block
constexpr int kJpegIdctUnroll = 4;                               // blocks per lane group
constexpr int kJpegIdctBlocks = kJpegIdctLanes / 8 * kJpegIdctUnroll; // blocks per IDCT workgroup (chunk)
constexpr int kJpegRowsPerWg = 32;  // output rows per colour workgroup (fewer when the staged rows outgrow LDS)
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
