// aug_job.hpp -- per-image work descriptors shared by the host planner (plan.cpp) and the
// HIP kernels (augment_kernels.hip).  One AugJob = one image's pass through
// crop -> [add_padding] -> resize -> cbsjitter -> lighting -> flip -> loader::load
// (aeon src/etl_image.cpp:146-202, 246-341), with every per-image constant that aeon
// derives on the host (cv::transform matrix, lighting pixel, cropbox) precomputed.
#pragma once
#include <stdint.h>

namespace aeon_hip {

enum ResizeMode : int32_t {
    RESIZE_COPY     = 0, // image::resize identity (size already matches, image.cpp:98-101)
    RESIZE_LINEAR   = 1, // cv::resize INTER_LINEAR, 11-bit fixed point
    RESIZE_AREA2X   = 2, // INTER_LINEAR at exactly 2x is routed to INTER_AREA's fast path
    RESIZE_NEAREST  = 3, // cv::resize INTER_NEAREST (pixel masks)
};

enum PhotoFlags : int32_t {
    PHOTO_BS       = 1, // brightness/saturation cv::transform
    PHOTO_HUE      = 2, // BGR->HSV8, H=(H+hue)%180, HSV8->BGR
    PHOTO_CONTRAST = 4, // x*c + (1-c)*mean(image)
    PHOTO_LIGHTING = 8, // (x + pca_pixel)/(1+sigma)
};

enum BsKind : int32_t { BS_DIAG = 0, BS_FIXPT = 1, BS_FLOAT = 2 };

// Output element types, AEON_DTYPE_* codes (aeon output_type -> cv type).
enum OutDtype : int32_t { OUT_U8 = 0, OUT_F32 = 1, OUT_S8 = 2, OUT_S16 = 3, OUT_U16 = 4, OUT_S32 = 5, OUT_F64 = 6 };

#if defined(__HIPCC__)
__host__ __device__
#endif
inline int out_elem_bytes(int dt)
{
    return dt == OUT_U8 || dt == OUT_S8 ? 1 : (dt == OUT_S16 || dt == OUT_U16 ? 2 : (dt == OUT_F64 ? 8 : 4));
}

// 16-byte aligned, plain data (copied H2D as an array).  Every field a tile of a launch without
// photometric stages reads lies in the first kJobHotBytes: such launches fetch only that half of
// each job (a single-pass call's tiles read their jobs over PCIe from the caller's pinned slot).
struct alignas(16) AugJob {
    double   scale_x, scale_y;  // OpenCV's 1/inv_scale (bilinear/nearest coefficient maths)
    uint64_t src_ptr;           // device address of the source image (HWC uint8)
    uint64_t src_bytes;         // bytes readable from src_ptr (buffer-descriptor range)
    uint64_t out_ptr;           // device address of the output item
    int32_t  src_stride, cn;
    int32_t  crop_x, crop_y, crop_w, crop_h; // region fed to the resize
    int32_t  shift_x, shift_y, padded;       // add_padding (image.cpp:77-91) as a virtual zero
                                             // border: resize-source (u,v) reads crop
                                             // (u+shift_x, v+shift_y), zero outside the crop
    int32_t  dst_w;                          // full resize target width
    int32_t  win_x, win_y, win_w, win_h;     // window of the target produced by this job
    int32_t  xv;                             // first element (x*cn+c) on OpenCV's scalar row tail
    int32_t  flip;
    int32_t  photo;                          // PhotoFlags
    int32_t  tiles;                          // row chunks (workgroups) of this job
    int32_t  stats_slot;                     // contrast partial-sum slot (-1 if none)
    int32_t  out_pitch, out_plane;           // loader output row pitch / plane stride (elements):
                                             // win_w / win_w*win_h, or the fixed_aspect_ratio canvas
    // -- photometric constants and host bookkeeping
    int32_t  mode;                           // ResizeMode
    int32_t  src_w, src_h, dst_h;
    int32_t  bs_kind;                        // BsKind
    int32_t  bsq[9];                         // 10-bit fixed-point transform coefficients
    float    bsm[9];                         // float transform matrix (diag / float paths)
    float    contrast;
    int32_t  hue;
    float    light_a;                        // (float)(1/(1+sigma))
    int32_t  light_add[3];                   // cvRound(pixel_c / (1+sigma))
    int32_t  src_scratch;                    // host bookkeeping: source lives in the slot scratch
    int32_t  stats_tiles;                    // chunks of the pass-1 job that wrote this slot's sums
};
constexpr int kJobHotBytes = 128;
static_assert(__builtin_offsetof(AugJob, mode) <= kJobHotBytes, "AugJob hot fields");
static_assert(sizeof(AugJob) == 256, "AugJob size");

// image::rotate pre-pass of one record (rotate_kernels.hip): source -> same-size scratch image.
struct alignas(16) RotJob {
    double   M[6];     // warpAffine's inverted affine map (output -> source), as OpenCV computes it
    uint64_t src_ptr;  // HWC uint8 source
    uint64_t out_ptr;  // HWC uint8 window [ox, ox+ow) x [oy, oy+oh) of the rotated image (ow * cn bytes per row)
    int32_t  w, h, stride, cn; // the source (= rotated image) size; cn = bytes per pixel (1..4)
    int32_t  interp;   // AEON_INTERP_LINEAR (images) or AEON_INTERP_NEAREST (pixel masks)
    int32_t  ox, oy, ow, oh; // the window of the rotated image later stages read (the cropbox, or all)
    int32_t  angle;          // degrees (sizes the launch's LDS source box)
    int32_t  pad_[2];
};

// image::expand pre-pass of one record (rotate_kernels.hip): the record at (ox, oy) of a zeroed
// ew x eh canvas in the slot scratch (src/image.cpp:276-303).
struct alignas(16) ExpandJob {
    uint64_t src_ptr;     // HWC uint8 record (its original, or its rotated copy in scratch)
    uint64_t out_ptr;     // HWC uint8 canvas, ew * cn bytes per row
    int32_t  w, h, stride, cn;
    int32_t  ew, eh, ox, oy;
    int32_t  src_scratch; // host bookkeeping: src_ptr / out_ptr are slot-scratch offsets until relocated
    int32_t  pad_[3];
};

// cv::resize with INTER_CUBIC / INTER_LANCZOS4 / INTER_AREA (aeon's interpolation_method, image.cpp:30-36)
// of one record: a pre-pass (resize_kernels.hip) writing the resized window as HWC uint8 into the slot
// scratch; the record's tile job then copies it (RESIZE_COPY) through the photometric stages and the
// loader.  GR_LINEAR_AREA is INTER_AREA's bilinear emulation when an axis is upscaled.
enum GrMethod : int32_t { GR_LINEAR_AREA = 0, GR_CUBIC = 1, GR_LANCZOS4 = 2, GR_AREA_FAST = 3, GR_AREA = 4 };
struct alignas(16) ResizeJob {
    double   scale_x, scale_y;  // OpenCV's 1 / inv_scale
    double   inv_x, inv_y;      // inv_scale = dst / src (area-mode coefficients)
    uint64_t src_ptr;           // HWC uint8: the record, or its rotated / expanded / resize_short copy
    uint64_t out_ptr;           // HWC uint8 window, win_w * cn bytes per row (slot scratch)
    int32_t  src_stride, cn;
    int32_t  crop_x, crop_y, crop_w, crop_h; // the region resized (cv::resize's source)
    int32_t  shift_x, shift_y, padded;       // add_padding as a virtual zero border (as AugJob)
    int32_t  dst_w, dst_h;                   // the full resize target
    int32_t  win_x, win_y, win_w, win_h;     // its window produced here
    int32_t  method;                         // GrMethod
    int32_t  isx, isy;                       // GR_AREA_FAST integer factors
    int32_t  coef_x, coef_y;                 // GR_LANCZOS4: host-built taps, byte offsets in the call's table
    int32_t  tiles_x, tiles;                 // column bands of the window, tiles in all
    int32_t  src_scratch, out_scratch;       // host bookkeeping: offsets into the slot scratch until relocated
    int32_t  final_out, flip;                // final_out: out_ptr is the loader's item (flip, standardize LUT,
    int32_t  out_pitch, out_plane;           // f32 planes or HWC at these strides), no copy pass after this one
};
// GR_LANCZOS4 taps per destination column / row as the host builds them (interpolateLanczos4 with
// the C library's sin / cos, as OpenCV): first source index, then 8 fixed-point coefficients.
struct GrTap {
    int32_t s;
    int16_t c[8];
};
// What the host computes per GR_LANCZOS4 destination column / row: the source anchor s and fraction f
// (cv::resize's), and sin / cos of y0 = -(f + 3) * pi / 4 from the C library, as OpenCV's
// interpolateLanczos4 takes them (imgwarp.cpp); the device finishes the eight coefficients
// (lanczos4_taps, resize_kernels.hip) in the same IEEE operations, so the taps are the host's bit for bit.
struct LzIn {
    double  s0, c0;
    float   f;
    int32_t s;
};

// Per-launch uniform arguments.
struct LaunchArgs {
    const AugJob*  jobs;       // the launch's jobs: device memory, or the device view of a pinned host slot
    int32_t        jobs_host;  // jobs is pinned host memory (read through to the host)
    int32_t        job_bytes;  // bytes of each job the tiles fetch: kJobHotBytes without photometric jobs
    int32_t        job_stride; // bytes between consecutive jobs of the table: sizeof(AugJob), or kJobHotBytes
                               // for a direct call's compact table of hot halves
    const float*   lut;        // [3][256] per SOURCE channel: standardized value of output
                               // channel (bgr_to_rgb ? 2-c : c), or (float)x without mean
    const int32_t* hsv_tables; // sdiv[256], hdiv180[256], then per uchar H the HSV2RGB weights (B, G, R, 0) as float bits
    uint32_t*      partials;   // contrast partial sums [slots][partial_stride][4]
    double*        shifts;     // contrast (1-c)*mean per slot [slots][4] (contrast_reduce)
    int32_t*       error;      // device error word (0 = ok)
    uint32_t*      trace;      // development only: per-workgroup phase timestamps (null = off)
    int32_t        rows_per_tile;  // output rows per tile (TR)
    int32_t        max_tiles;      // tiles per job (tile t = band t % max_tiles of job t / max_tiles)
    int32_t        total_tiles;    // jobs * max_tiles
    int32_t        stage_bytes;    // capacity of one LDS staging buffer (multiple of 1 KiB)
    int32_t        max_win_w;  // capacity of the column-tap tables
    int32_t        out_dtype;  // OutDtype
    int32_t        channel_major;
    int32_t        bgr_to_rgb;
    int32_t        vec_ok;     // outputs 16-byte aligned and win_w % 4 == 0 for every job
    int32_t        lds_bytes;
    int32_t        has_hue;    // some job of the launch shifts hue (HSV tables in LDS)
    int32_t        partial_stride; // (tile, wave) entries per contrast slot in `partials`
    int32_t        threads;    // workgroup size (kBlockMin..kBlockMax, a multiple of 64)
    int32_t        has_rtab;   // LDS holds a per-record table (contrast -> lighting -> standardize)
    int32_t        u8_map;     // uint8 stores go through the LUT (fixed_aspect_ratio's uint8 standardize)
    int32_t        has_mean;   // double output: standardize with smean / sinv (by SOURCE channel)
    uint32_t*      tail_ctr;   // non-null: the partial last round of tiles is handed out by this counter
                               // (zero on entry; the launch's last draw resets it)
    int32_t        tail_rounds; // ... and this many full rounds before it
    // image + mask calls (aeon_hip_augment_pair_batch): the masks' NEAREST row blocks, which the
    // launch's workgroups draw from m_ctr after their tiles (mask16_device.hpp; 0 blocks: none)
    const struct Mask16Job* mjobs;
    uint32_t*      m_ctr;      // zero on entry; the launch's last draw resets it
    int32_t        m_blocks;   // m_jobs x m_bpj row blocks
    int32_t        m_bpj;      // row blocks per mask (m_rows output rows each)
    int32_t        m_rows, m_pitch, m_perm, m_slots; // nearest_staged's geometry (launch_nearest)
    int32_t        m_lds;      // LDS byte offset of the blocks' row map, job and staged rows
    double         smean[3], sinv[3]; // sinv = 1/stddev, or 0 for stddev 0 (no division)
};

// KM_FINAL: a record through to the loader output.  KM_STATS: contrast pass 1 -- resize +
// brightness/saturation + hue into an HWC uint8 intermediate plus exact per-chunk channel sums
// (the mean cv::mean needs).  KM_RAW: resize only, HWC uint8 (resize_short pre-pass).
enum KernelMode : int { KM_FINAL = 0, KM_STATS = 1, KM_RAW = 2 };

// Workgroups are 256..512 lanes: a multiple of the window's 4-pixel column groups, so every
// lane keeps the same output columns (and their resize taps) for a whole chunk.
constexpr int kBlockMin = 256;
constexpr int kBlockMax = 512;
constexpr int kHsvWords = 512 + 256 * 4; // RGB2HSV division tables + HSV2RGB per-H weights (global copy)
constexpr int kHsvDivWords = 512;         // ... of which the division tables (sdiv, hdiv180)
// In LDS: per v {sdiv[v], bits of (float)v * (1.f / 255)} (8 B, one read gives the HSV2RGB v too),
// then hdiv180[256], then the per-tile hue tables.
constexpr int kHsvLdsDivBytes = 256 * 8 + 256 * 4;
// Per tile of a hue record, in LDS: the HSV2RGB weights of the record's shifted H for every
// OpenCV h before its +180 wrap, h12 in [-30, 150] (tools/hue_range.py): entry h12 + 30 holds
// weights[((h12 < 0 ? h12 + 180 : h12) + hue) % 180 as uchar], so the pixel loop does one lookup.
constexpr int kHueTabEntries = 181;
constexpr int kHueTabBytes   = 184 * 16;

#if defined(__HIPCC__)
#define AEON_HD __host__ __device__
#else
#define AEON_HD
#endif

// LDS bytes of a staged source of `rows` rows x `cols` columns (augment_kernels.hip stage_need): the
// rows' units back to back in whole 64-unit DMA instructions -- BGR groups of 4 pixels as 16-byte
// slots (1 KiB per instruction), or gray pixels as words (256 B per instruction).
AEON_HD inline long stage_bytes_for(int cn, int rows, int cols)
{
    const long groups = (long)rows * ((cols + 3) / 4);
    return cn == 3 ? (groups + 63) / 64 * 1024 : (groups * 4 + 63) / 64 * 256;
}

// LDS carve of one workgroup (bytes; every region 16-byte aligned, see the CDNA guide G17).
struct LdsLayout {
    int lut, hsv, rtab, xt, yt, job, info, stage, stage_bytes, total;
};
// One staging buffer and the tap tables.  The HSV tables are reserved only for hue launches.  The
// LUT sits at offset 0 so its per-channel reads use immediate LDS offsets.
AEON_HD inline LdsLayout lds_layout(int max_win_w, int rows_per_tile, int stage_bytes, bool hue, bool rtab = false)
{
    LdsLayout L;
    int       o = 0;
    L.lut = o; o += 3 * 256 * 4;                             // standardize LUT (source channel order)
    L.hsv = o; o += hue ? kHsvLdsDivBytes + kHueTabBytes : 0; // sdiv + v/255 / hdiv180, per-tile hue tables
    L.rtab = o; o += rtab ? 3 * 256 * 4 : 0;                 // the tile's record table (f32, source channel order)
    L.xt  = o; o += ((max_win_w * 8 + 15) / 16) * 16; // per-column taps + weights
    L.yt  = o; o += rows_per_tile * 16;               // per-row taps + weights
    L.job = o; o += 3 * (int)sizeof(AugJob);                 // a ring of three tiles' jobs (LDS-DMA copies)
    L.info = o; o += 64;                                     // the next tile's geometry (one wave computes it)
    L.stage_bytes = stage_bytes;                             // source pixels, 4 B each (B,G,R,x)
    L.stage = o; o += stage_bytes;
    L.total = o;
    return L;
}

// ---- split_kernels.hip: the single-pass tile kernel with staging helper waves ----------------------
// LDS carve of augment_split (bytes, 16-aligned regions): the LUT at offset 0 (lut_at), then per
// staging buffer b its column taps, row taps and tile info, a ring of jobs, the staging buffers.  Three
// buffers: the compute waves work on tile k while tile k + 1 is unpacked and tile k + 2's loads are in
// flight (a tile's LDS-DMA then has a whole tile's time to land).
constexpr int kSplitBufs   = 3;  // staging buffers
constexpr int kSplitTRMax  = 64; // output rows per tile, at most (row-tap table size)
constexpr int kSplitJobs   = 6;  // job ring slots: tiles k (compute), k + 1 (unpack), k + 2 (issue), k + 3 (geometry),
                                 // k + 4 (landed), k + 5 (fetched)
constexpr int kSplitGeo    = 4;  // tile geometry slots: tiles k, k + 1, k + 2, k + 3
struct SplitLds {
    int lut, xt, yt, job, info, stage, stage_bytes, xt_bytes, total;
};
AEON_HD inline SplitLds split_lds_layout(int win_w, int stage_bytes)
{
    SplitLds L;
    int      o = 0;
    L.lut = o; o += 3 * 256 * 4;                         // standardize LUT (source channel order)
    L.xt_bytes = ((win_w * 8 + 15) / 16) * 16;
    L.xt  = o; o += kSplitBufs * L.xt_bytes;             // column taps + weights, per buffer
    L.yt  = o; o += kSplitBufs * kSplitTRMax * 16;       // row taps + weights, per buffer
    L.job = o; o += kSplitJobs * (int)sizeof(AugJob);    // the jobs of six consecutive tiles
    L.info = o; o += kSplitGeo * 64;                     // per tile of the ring: its geometry (split_kernels.hip)
    L.stage_bytes = stage_bytes;
    L.stage = o; o += kSplitBufs * stage_bytes;          // the staging buffers
    L.total = o;
    return L;
}
struct SplitArgs {
    int nwc;   // compute waves (the first nwc * 64 lanes); the rest of the workgroup stages
    int nph;   // row phases of the compute lanes (nph * win_w / 4 <= nwc * 64)
    int rpl;   // output rows per compute lane per tile: rows_per_tile = nph * rpl
    int win_w; // the launch's common window width (a multiple of 4)
    int occ;   // workgroups per CU (1 or 2: the kernel's register budget; host only)
};

// ---- record_kernels.hip: contrast records in one launch (the post-hue record in registers) ------
constexpr int kRecPhasesMax = 32;                  // row phases (lanes per column group), at most
constexpr int kRecRows   = 14;                     // rows per lane held in registers (win_h <= 224)
constexpr int kRecTileRows = 2;                    // rows per lane per tile
constexpr int kRecTRMax  = kRecPhasesMax * kRecTileRows; // output rows per tile (2 x phases), at most
constexpr int kRecTiles  = kRecRows / kRecTileRows;   // register tiles (the rotation period)
constexpr int kRecWords  = 3 * kRecRows;           // 12 bytes (4 BGR pixels) per row

// LDS carve of the record kernel (bytes, 16-aligned regions)
struct RecLds {
    int rtab, lut, hwt, hsv, htab, xt, xt2, yt, job, sums, flags, stage, stage_bytes, total;
};
AEON_HD inline RecLds rec_lds_layout(int win_w, int stage_bytes)
{
    RecLds L;
    int    o = 0;
    L.rtab = o; o += 3 * 256 * 4;           // record table of the B record (f32, source channel order)
    L.lut  = o; o += 3 * 256 * 4;           // the launch's standardize LUT (record tables read it)
    L.hwt  = o; o += 256 * 16;              // HSV2RGB weights per uchar H (hue tables read them)
    L.hsv  = o; o += kHsvLdsDivBytes;       // sdiv + v/255, hdiv180
    L.htab = o; o += kHueTabBytes;          // hue table of the A record
    L.xt   = o; o += ((win_w * 8 + 15) / 16) * 16; // column taps of the A record
    L.xt2  = o; o += ((win_w * 8 + 15) / 16) * 16; // (plain_records: the next record's)
    L.yt   = o; o += 2 * kRecTRMax * 16;    // row taps, one table per staging buffer
    L.job  = o; o += 3 * (int)sizeof(AugJob); // a ring of three records' jobs
    L.sums = o; o += 16 * 16;               // per-wave channel sums
    L.flags = o; o += 16;                   // (split kernel) staging buffer b's tile is valid: word b
    L.stage_bytes = stage_bytes;
    L.stage = o; o += 2 * stage_bytes;      // two staging buffers
    L.total = o;
    return L;
}

// Row phases of a win_w-wide record: 16 (a 224-wide record on 16 x 56 = 896 lanes, 14 waves: measured
// 262 us per C3 batch against 271-275 us with 18 phases, 1,008 lanes) when the lanes' registers then
// hold win_h rows (kRecRows per lane), else as many as 1024 lanes allow (at most kRecPhasesMax); 0 if
// no lane count holds the record.
AEON_HD inline int rec_phases(int win_w, int win_h)
{
    const int gpr = win_w / 4;
    if (gpr <= 0) return 0;
    const int most = 1024 / gpr < kRecPhasesMax ? 1024 / gpr : kRecPhasesMax;
    const int nph  = most >= 16 && (win_h + 15) / 16 <= kRecRows ? 16 : most;
    return nph > 0 && (win_h + nph - 1) / nph <= kRecRows ? nph : 0;
}

struct RecArgs {
    int n_jobs;    // records of the launch
    int phases;    // row phases (rec_phases)
    int win_w, win_h; // output size of every record (win_w % 4 == 0, win_w <= 256, win_h <= 224)
    int tiles;     // tiles per record = ceil(rows per lane / 2)
};

} // namespace aeon_hip
