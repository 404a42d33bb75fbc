// stage.cpp -- host side of the HIP augmentation stage: per-record planning (the host-side
// arithmetic aeon does per record before touching pixels), the per-GPU context with its
// pinned/device staging ring, kernel launches and the extern "C" boundary (include/aeon_hip.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/aeon_hip.h"
#include "aug_job.hpp"
#include "host.hpp"
#include "jpeg.hpp"
#include "mask16.hpp"
#include "json.hpp"
#include "param_factory.hpp"
#include "plan_record.hpp"

namespace aeon_hip {
hipError_t launch_tiles(int km, int rm, bool tail, bool photo, const LaunchArgs& a, int grid, hipStream_t stream,
                        hipEvent_t start, hipEvent_t stop);
hipError_t launch_contrast_reduce(const LaunchArgs& a, int n_jobs, hipStream_t stream);
hipError_t kernel_occupancy(int km, int rm, bool tail, bool photo, const LaunchArgs& a, int* blocks);
hipError_t set_kernel_lds_limit(int bytes);
hipError_t launch_transpose(const void* src, void* dst, int64_t rows, int64_t cols, int element_size,
                            hipStream_t stream);
hipError_t launch_rotate(const RotJob* jobs, int n_jobs, int max_tiles, int words, int cn, int32_t* error,
                         hipStream_t stream);
int        rot_box_words(int angle);
hipError_t launch_expand(const ExpandJob* jobs, int n_jobs, int max_pixels, hipStream_t stream);
hipError_t launch_nearest(const Mask16Job* jobs, int n_jobs, int max_h, int max_w, int max_seg_bytes, int max_slots, hipStream_t stream,
                          hipEvent_t start, hipEvent_t stop);
hipError_t launch_upload_table(const void* host_dev, void* dst, size_t bytes, hipStream_t stream);
hipError_t launch_contrast_records(bool fast, bool split, const LaunchArgs& a, const RecArgs& r, int grid, hipStream_t stream,
                                   hipEvent_t start, hipEvent_t stop);
hipError_t contrast_records_lds_limit(int bytes);
hipError_t launch_split(bool tail, int occ, const LaunchArgs& a, const SplitArgs& s, int grid, hipStream_t stream,
                        hipEvent_t start, hipEvent_t stop);
hipError_t split_lds_limit(int bytes);
hipError_t split_occupancy(bool tail, int occ, const LaunchArgs& a, int* blocks);
hipError_t launch_resize_generic(const ResizeJob* jobs, const uint8_t* table, int n_jobs, int max_tiles, int TR, int CW,
                                 int NR, int xs, int amax, int cn_max, int SW, const float* lut, int bgr, int chm,
                                 int32_t* error, hipStream_t stream);
hipError_t launch_lanczos4_taps(const LzIn* in, GrTap* out, int n, hipStream_t stream);
hipError_t launch_resize_sep(int K, bool area, const ResizeJob* jobs, const uint8_t* table, int n_jobs, int max_tiles, int TR, int CW,
                             int NR, int SW, int cn, const float* lut, int bgr, int chm, int32_t* error, hipStream_t stream);
void       jpeg_decode_batch(JpegState* S, int n, const void* const* data, const size_t* sizes,
                             const aeon_img_desc* descs, void* dst_base, int32_t* error, hipStream_t stream,
                             hipEvent_t start, hipEvent_t stop);
void       jpeg_info(const void* data, size_t size, int* w, int* h, int* ncomp);
void       jpeg_entropy_only(const void* data, size_t size, int* w, int* h, int* ncomp, int64_t* n_blocks,
                             int64_t* n_values, uint64_t* hash);
void       jpeg_host_stage(const void* data, size_t size, int* gpu_entropy, int64_t* staged_bytes);
void       png_header(const void* data, size_t size, int* w, int* h, int* depth, int* ctype);
void       png_decode(const void* data, size_t size, int mode, void* dst, size_t stride, int* out_elem_bytes);
} // namespace aeon_hip

using namespace aeon_hip;

namespace {

thread_local std::string g_err;

struct aeon_error : std::runtime_error {
    int code;
    aeon_error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
[[noreturn]] void fail(int code, const std::string& msg) { throw aeon_error(code, msg); }

// The device error word's bits (kernels atomicOr them; aeon_hip_synchronize reports and clears).
std::string device_error_text(int err)
{
    static const struct {
        int         bit;
        const char* what;
    } bits[] = {{2, "LDS staging footprint exceeded"},
                {4, "dynamic LDS not at address 0"},
                {16, "hue table without a t1 channel"},
                {32, "dynamic-tail counter left over by an earlier launch"},
                {64, "rotation source box exceeds the launch's LDS"},
                {128, "generic resize footprint exceeds the launch's LDS"},
                {256, "JPEG entropy-coded data corrupt or truncated (GPU Huffman decoder)"},
                {512, "separable resize band wider than its workgroup"}};
    std::string s;
    for (const auto& b : bits)
        if (err & b.bit) s += (s.empty() ? "" : "; ") + std::string(b.what);
    return s.empty() ? "unknown" : s;
}

#define HIP_OK(expr)                                                                           \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) fail(AEON_HIP_ERUNTIME, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kMaxLds        = 160 * 1024;
// launch-shape constants (compile-time overrides only for tuning builds, tools/build_variants.sh)
#ifndef AEON_HIP_STAGE_BUDGET_KB
#define AEON_HIP_STAGE_BUDGET_KB 48
#endif
#ifndef AEON_HIP_FIXED_THREADS
#define AEON_HIP_FIXED_THREADS 0
#endif
constexpr int kStageBudget   = AEON_HIP_STAGE_BUDGET_KB * 1024; // preferred LDS bytes of the staging buffer
constexpr int kStageBudgetHi = 140 * 1024;  // fallback for very wide crops
#ifndef AEON_HIP_UPLOAD_KERNEL_MAX_KB
#define AEON_HIP_UPLOAD_KERNEL_MAX_KB 128
#endif
constexpr size_t kUploadKernelMax = AEON_HIP_UPLOAD_KERNEL_MAX_KB * 1024; // job tables above this go up by SDMA (run_batch)
constexpr size_t kDirectFetchMax  = 512 * 1024; // run_direct: most job bytes a launch's tiles read over PCIe

// ---------------------------------------------------------------------------------------------
// Per-image constants (aeon computes these on the host per record, too)
// ---------------------------------------------------------------------------------------------

// image::standardize arithmetic (src/image.cpp:129-174 over OpenCV 2.4 arithm_op: f64 work
// type per op, rounded to f32 after each op) tabulated per channel and input value.
void build_lut(const aeon_out_desc& o, float* lut, bool u8_map = false)
{
    if (u8_map) {
        // fixed_aspect_ratio's in-place standardize of its uint8 canvas (etl_image.cpp:263-300 ->
        // image.cpp:129-174 on CV_8U planes): OpenCV 2.4 arithm_op on 8U -- multiply(1/255.) in
        // double, subtract the mean converted to int (cvRound, add/sub rule), multiply(1/stddev)
        // in double -- each saturated to uint8
        for (int c = 0; c < 3; c++) {
            const int oc = (o.bgr_to_rgb && o.channels == 3) ? 2 - c : c;
            for (int x = 0; x < 256; x++) {
                if (oc >= o.channels) {
                    lut[c * 256 + x] = (float)x;
                    continue;
                }
                auto sat = [](int v) { return std::min(std::max(v, 0), 255); };
                int  a   = sat(cv_round((double)x * (1. / 255.)));
                a        = sat(a - cv_round(o.mean[oc]));
                if (o.stddev[oc] != 0) a = sat(cv_round((double)a * (1. / o.stddev[oc])));
                lut[c * 256 + x] = (float)a;
            }
        }
        return;
    }
    // indexed by SOURCE channel c; its value lands in output channel oc (mixChannels
    // from_to {0,2,1,1,2,0} when bgr_to_rgb), standardized with that channel's mean/stddev
    for (int c = 0; c < 3; c++) {
        const int oc = (o.bgr_to_rgb && o.channels == 3) ? 2 - c : c;
        for (int x = 0; x < 256; x++) {
            if (!o.has_mean || oc >= o.channels) {
                lut[c * 256 + x] = (float)x;
                continue;
            }
            float t1 = (float)((double)(float)x * (1. / 255.));
            float t2 = (float)((double)t1 - o.mean[oc]);
            lut[c * 256 + x] = o.stddev[oc] != 0 ? (float)((double)t2 * (1. / o.stddev[oc])) : t2;
        }
    }
}

// What the launch planner needs to know of a job (the fields share AugJob's names, so the
// templates below take either).
struct JobGeom {
    int32_t mode, cn, crop_w, crop_h, win_w, win_h, dst_w, dst_h, photo, stats_slot;
    double  scale_x, scale_y;
};

// source-footprint bounds used to size the LDS staging area
template <typename J_>
int stage_cols(const J_& J)
{
    switch (J.mode) {
    // +1: the second tap column is staged even where its weight is 0
    case RESIZE_LINEAR: return std::min(J.crop_w + 1, (int)std::ceil((J.win_w - 1) * J.scale_x) + 4);
    case RESIZE_NEAREST: return std::min(J.crop_w, (int)std::ceil((J.win_w - 1) * J.scale_x) + 3);
    case RESIZE_AREA2X: return 2 * J.win_w;
    default: return J.win_w;
    }
}
template <typename J_>
int stage_rows_for(const J_& J, int tr)
{
    int rows = std::min(tr, J.win_h);
    switch (J.mode) {
    case RESIZE_LINEAR: return std::min(J.crop_h, (int)std::ceil((rows - 1) * J.scale_y) + 3);
    case RESIZE_NEAREST: return std::min(J.crop_h, (int)std::ceil((rows - 1) * J.scale_y) + 2);
    case RESIZE_AREA2X: return 2 * rows;
    default: return rows;
    }
}

struct LaunchPlan {
    int                 rm = RESIZE_LINEAR;
    bool                photo = false;
    bool                tail  = false; // LINEAR jobs with OpenCV scalar-tail columns
    size_t              blob_off = 0;     // byte offset of this group's jobs in the slot blob
    std::vector<AugJob> jobs;
    int                 tr = 1, stage_bytes = 0, max_win_w = 0, max_tiles = 0;
    int                 lds = 0, threads = kBlockMax;
    bool                vec_ok = true;
    bool                has_hue = false, has_contrast = false;
    bool                rtab    = false; // final f32 launch with contrast / lighting: per-record LDS table
    bool                split   = false; // launched as augment_split (shape set by plan_split)
    SplitArgs           sa{};

    // launch shape for this->jobs (unless plan_split set it), and each job's tile count
    void finalize()
    {
        if (jobs.empty()) return;
        if (!split) shape(jobs);
        max_tiles = 0;
        for (AugJob& J : jobs) {
            J.tiles   = (J.win_h + tr - 1) / tr;
            max_tiles = std::max(max_tiles, J.tiles);
        }
    }

    // workgroup size, rows per tile, LDS staging size for a set of jobs (AugJob or JobGeom)
    template <typename J_>
    void shape(const std::vector<J_>& jobs)
    {
        int ww = 0;
        for (const J_& J : jobs) ww = std::max(ww, J.win_w);
        max_win_w = std::max(ww, 1);
        // workgroup = 256..512 lanes holding whole 4-pixel column groups (fewest idle lanes;
        // ties go to the larger group), row phases = lanes / column groups
        const int gpr = (max_win_w + 3) / 4;
        const int ncg = std::min(gpr, kBlockMax);
        threads       = kBlockMax;
        int best_idle = kBlockMax;
        for (int nt = kBlockMin; nt <= kBlockMax; nt += 64) {
            const int idle = nt - (nt / ncg) * ncg;
            // idle / nt <= best_idle / threads
            if ((long)idle * threads <= (long)best_idle * nt) threads = nt, best_idle = idle;
        }
        // contrast pass 2 (photometric over the u8 intermediate, no resize): full workgroups
        // beat the fewest-idle-lanes choice (C3: 140 vs 158 us at 512 vs 448 lanes)
        if (rm == RESIZE_COPY && photo) threads = kBlockMax;
        if (AEON_HIP_FIXED_THREADS) threads = AEON_HIP_FIXED_THREADS;
        const int nph = threads / ncg;
        // one staging buffer and four rows per lane (a multiple of the row phases): the CU's other
        // workgroups cover a tile's staging latency.  Measured on C2/C3 against two buffers
        // (the next tile's loads in flight during the current tile's compute) at two rows per
        // lane: 42 vs 45 us (C2), 152/291 vs 186/370 us (C3 pass 2 / pass 1) -- the second
        // buffer costs occupancy and halves the rows per tile (rejected).
        // (development: AEON_HIP_TILE_ROWS caps the rows per tile instead)
        static const int tr_env = std::getenv("AEON_HIP_TILE_ROWS") ? std::atoi(std::getenv("AEON_HIP_TILE_ROWS")) : 0;
        const int        tr_cap = std::min(64, std::max(1, tr_env > 0 ? tr_env : 4 * nph));
        int       budget = kStageBudget;
        bool hue = false, contrast = false;
        for (const J_& J : jobs) {
            hue |= (J.photo & PHOTO_HUE) != 0;
            contrast |= (J.photo & PHOTO_CONTRAST) != 0 && J.stats_slot >= 0;
        }
        has_hue = hue, has_contrast = contrast;
        for (int pass = 0; pass < 2; pass++) {
            for (int t = tr_cap; t >= 1; t--) {
                // staged rows, each in whole DMA instructions (stage_bytes_for)
                long by = 0;
                for (const J_& J : jobs) by = std::max(by, stage_bytes_for(J.cn, stage_rows_for(J, t), stage_cols(J)));
                by = (by + 1023) / 1024 * 1024;
                if (by <= budget || (t == 1 && pass == 1)) {
                    tr = t, stage_bytes = (int)by;
                    goto chosen;
                }
            }
            budget = kStageBudgetHi;
        }
    chosen:
        lds = lds_layout(max_win_w, tr, stage_bytes, photo && hue, rtab).total;
        if (lds > kMaxLds)
            fail(AEON_HIP_EUNSUPPORTED, "source crop too wide for LDS-staged row bands (" + std::to_string(lds) +
                                            " bytes)");
    }
};

// Geometry + constants of one image-provider record (transform_single_image).
// image::rotate (src/image.cpp:53-75): cv::getRotationMatrix2D(Point2i(cols/2, rows/2), angle, 1)
// inverted the way cv::warpAffine does without WARP_INVERSE_MAP (OpenCV 2.4 imgwarp.cpp); double
// arithmetic on the host, as aeon's.
void rotation_inverse_map(int w, int h, int angle, double M[6])
{
    const float  cx = (float)(w / 2), cy = (float)(h / 2); // Point2i -> Point2f
    const double a  = (double)angle * (3.1415926535897932384626433832795 / 180);
    const double alpha = std::cos(a) * 1.0, beta = std::sin(a) * 1.0;
    M[0] = alpha, M[1] = beta, M[2] = (1 - alpha) * cx - beta * cy;
    M[3] = -beta, M[4] = alpha, M[5] = beta * cx + (1 - alpha) * cy;
    double D = M[0] * M[4] - M[1] * M[3];
    D        = D != 0 ? 1. / D : 0;
    const double A11 = M[4] * D, A22 = M[0] * D;
    M[0] = A11;
    M[1] *= -D;
    M[3] *= -D;
    M[4] = A22;
    const double b1 = -M[0] * M[2] - M[1] * M[5];
    const double b2 = -M[3] * M[2] - M[4] * M[5];
    M[2] = b1, M[5] = b2;
}

// A single-channel pixel-mask / depth-map record, 16-bit (CV_16U, ANYDEPTH) or rotation-free
// 8-bit: crop -> INTER_NEAREST -> flip -> convertTo (etl_pixel_mask.cpp:65-92,
// etl_depthmap.cpp:65-96, image.cpp:176-212), one gather pass (mask16_kernels.hip).
void rotation_inverse_map(int w, int h, int angle, double M[6]);

void plan_mask16(const aeon_img_desc& d, const void* src_base, const aeon_aug_params& p, const aeon_out_desc& o,
                 uint8_t* out_item, bool is_mask, std::vector<Mask16Job>& m16, std::vector<RotJob>& rot,
                 size_t& scratch_bytes)
{
    const int eb = d.elem_bytes == 2 ? 2 : 1;
    if (!is_mask) fail(AEON_HIP_EUNSUPPORTED, "16-bit sources are implemented for pixel masks / depth maps only");
    if (d.channels != 1 || o.channels != 1) fail(AEON_HIP_EINVAL, "16-bit masks must have one channel");
    if (d.width <= 0 || d.height <= 0 || d.stride < d.width * eb || (eb == 2 && ((d.stride & 1) || (d.offset & 1))))
        fail(AEON_HIP_EINVAL, eb == 2 ? "invalid 16-bit source image descriptor" : "invalid source image descriptor");
    if (p.out_w <= 0 || p.out_h <= 0) fail(AEON_HIP_EINVAL, "invalid output size");
    const size_t elem = out_elem_bytes(o.dtype);
    if ((size_t)p.out_w * p.out_h * elem > o.item_stride) fail(AEON_HIP_EINVAL, "output item does not fit item_stride");
    if (o.fixed_aspect_ratio && (p.out_w > o.canvas_w || p.out_h > o.canvas_h))
        fail(AEON_HIP_EINVAL, "fixed_aspect_ratio: output_size larger than the image canvas");
    if (p.crop_x < 0 || p.crop_y < 0 || p.crop_w <= 0 || p.crop_h <= 0 || p.crop_x + p.crop_w > d.width ||
        p.crop_y + p.crop_h > d.height)
        fail(AEON_HIP_EINVAL, "cropbox outside image");
    Mask16Job M{};
    M.scale_x    = 1. / ((double)p.out_w / p.crop_w);
    M.scale_y    = 1. / ((double)p.out_h / p.crop_h);
    M.src_ptr    = (uint64_t)((const uint8_t*)src_base + d.offset);
    M.out_ptr    = (uint64_t)out_item;
    M.src_stride = d.stride;
    M.crop_x = p.crop_x, M.crop_y = p.crop_y, M.crop_w = p.crop_w, M.crop_h = p.crop_h;
    M.out_w = p.out_w, M.out_h = p.out_h;
    M.out_pitch = o.fixed_aspect_ratio ? o.canvas_w : p.out_w;
    M.flip      = p.flip ? 1 : 0;
    M.dtype     = o.dtype;
    M.src_elem  = eb;
    if (p.angle != 0) {
        // image::rotate(..., interpolate = false, border 0) (etl_pixel_mask.cpp:72-74,
        // etl_depthmap.cpp:72-73): nearest moves whole elements, so a 16-bit record rotates as a
        // 2-byte-per-pixel one; the gather pass then reads the rotated copy in the slot scratch
        // only the cropbox window of the rotated record is produced (the gather reads nothing else)
        RotJob R{};
        rotation_inverse_map(d.width, d.height, p.angle, R.M);
        R.src_ptr = M.src_ptr;
        R.w = d.width, R.h = d.height, R.stride = d.stride, R.cn = eb;
        R.interp      = AEON_INTERP_NEAREST;
        R.ox = p.crop_x, R.oy = p.crop_y, R.ow = p.crop_w, R.oh = p.crop_h;
        size_t off    = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)R.ow * R.oh * eb + 16;
        R.out_ptr     = off; // relocated to the slot's scratch by the caller
        R.angle       = p.angle;
        rot.push_back(R);
        M.src_ptr     = off;
        M.src_scratch = 1;
        M.src_stride  = R.ow * eb;
        M.crop_x = M.crop_y = 0;
    }
    m16.push_back(M);
}

// Checks of one 8-bit record aeon's transformer would throw on (or that this stage refuses).
void validate_record(const aeon_img_desc& d, const aeon_aug_params& p, const aeon_out_desc& o, bool is_mask)
{
    const int cn = d.channels;
    if (cn != 1 && cn != 3) fail(AEON_HIP_EINVAL, "channels must be 1 or 3");
    if (cn != o.channels) fail(AEON_HIP_EINVAL, "decoded channels do not match the output config");
    if (d.width <= 0 || d.height <= 0 || d.stride < d.width * cn)
        fail(AEON_HIP_EINVAL, "invalid source image descriptor");
    const int interp = is_mask ? AEON_INTERP_NEAREST : p.interp;
    if (interp < AEON_INTERP_LINEAR || interp > AEON_INTERP_LANCZOS4) fail(AEON_HIP_EINVAL, "unknown interpolation");
    if (p.out_w <= 0 || p.out_h <= 0) fail(AEON_HIP_EINVAL, "invalid output size");
    const size_t elem = out_elem_bytes(o.dtype);
    if ((size_t)p.out_w * p.out_h * cn * elem > o.item_stride)
        fail(AEON_HIP_EINVAL, "output item does not fit item_stride");
    if (o.fixed_aspect_ratio && (p.out_w > o.canvas_w || p.out_h > o.canvas_h))
        fail(AEON_HIP_EINVAL, "fixed_aspect_ratio: output_size larger than the image canvas");
    int base_w = d.width, base_h = d.height;
    if (!is_mask && expands(p)) { // image::expand throws on a record that does not fit the canvas
        if (p.expand_x < 0 || p.expand_y < 0 || p.expand_x + d.width > p.expand_w || p.expand_y + d.height > p.expand_h)
            fail(AEON_HIP_EINVAL, "Invalid parameters to expand image");
        base_w = p.expand_w, base_h = p.expand_h;
    }
    if (!is_mask && p.resize_short_size > 0) get_resized_short_size(base_w, base_h, p.resize_short_size, &base_w, &base_h);
    if (p.crop_x < 0 || p.crop_y < 0 || p.crop_w <= 0 || p.crop_h <= 0 || p.crop_x + p.crop_w > base_w ||
        p.crop_y + p.crop_h > base_h)
        fail(AEON_HIP_EINVAL, (is_mask || p.resize_short_size <= 0) && !(!is_mask && expands(p))
                                  ? "cropbox outside image"
                                  : "cropbox outside the expanded / resize_short image");
    if (!is_mask && photo_flags(p) && cn != 3) fail(AEON_HIP_EINVAL, "photometric augmentation needs a 3-channel image");
    if (!is_mask && (p.n_lighting != 0 && p.n_lighting != 3)) fail(AEON_HIP_EINVAL, "lighting needs 3 values");
}

OutGeom out_geom(const aeon_out_desc& o) { return OutGeom{o.fixed_aspect_ratio, o.canvas_w, o.canvas_h}; }

// The cv::resize of a (sw x sh -> dw x dh) resize with interpolation `interp` when the tile kernel
// has no mode for it: a resize_generic method (CUBIC, LANCZOS4, INTER_AREA but its exact 2x box), or
// -1 -- LINEAR / NEAREST, any identity (every method reproduces the source at scale 1) and INTER_AREA's
// 2x fast path (RESIZE_AREA2X, the same (a+b+c+d+2)>>2).  OpenCV 2.4.9 cv::resize's dispatch.
int generic_method(int sw, int sh, int dw, int dh, int interp, int cn, int* isx, int* isy)
{
    if (interp != AEON_INTERP_CUBIC && interp != AEON_INTERP_AREA && interp != AEON_INTERP_LANCZOS4) return -1;
    if (sw == dw && sh == dh) return -1;
    if (interp == AEON_INTERP_CUBIC) return GR_CUBIC;
    if (interp == AEON_INTERP_LANCZOS4) return GR_LANCZOS4;
    const double sx = 1. / ((double)dw / sw), sy = 1. / ((double)dh / sh);
    if (sx < 1 || sy < 1) return GR_LINEAR_AREA; // an upscaled axis: bilinear over area-mode coefficients
    const int ix = cv_round(sx), iy = cv_round(sy);
    if (std::fabs(sx - ix) < DBL_EPSILON && std::fabs(sy - iy) < DBL_EPSILON) {
        if (ix == 2 && iy == 2 && (cn == 1 || cn == 3)) return -1;
        *isx = ix, *isy = iy;
        return GR_AREA_FAST;
    }
    return GR_AREA;
}

// The host half of interpolateLanczos4 (OpenCV 2.4.9 imgwarp.cpp) for destinations [d0, d0 + n) of an
// ssize -> dsize axis (x: the anchor clamped as cv::resize does for columns; y: raw, the rows clipped
// per tap on use): the anchor, the fraction and the double sin / cos of the C library as OpenCV's --
// the one part a device could not reproduce bit for bit.  The coefficients are finished on the device
// (lanczos4_taps, resize_kernels.hip).
void lanczos4_inputs(int ssize, double scale, int d0, int n, bool clamp, LzIn* out)
{
    const double kPi = 3.1415926535897932384626433832795;
    for (int d = d0; d < d0 + n; d++) {
        float f = (float)((d + 0.5) * scale - 0.5);
        int   s = (int)std::floor(f);
        f -= (float)s;
        if (clamp && s < 0) f = 0, s = 0;
        if (clamp && s >= ssize - 1) f = 0, s = ssize - 1;
        LzIn L{0.0, 0.0, f, s};
        if (!(f < FLT_EPSILON)) {
            // sin / cos of a function of the float f alone: memoised per thread.  A batch's fractions are
            // few (integer crop sizes over a common output size: multiples of 1 / (2 * size), rounded to
            // float), so a 256-record LANCZOS4 call computes a few thousand pairs instead of 115 K (the
            // host side was the C2:LANCZOS4 step's bound).  Same libm calls on the same doubles: the
            // same bits.
            struct Entry {
                uint32_t key; // float bits + 1 (0: empty)
                double   s, c;
            };
            static thread_local std::vector<Entry> memo(1 << 14);
            uint32_t bits;
            std::memcpy(&bits, &f, 4);
            Entry& e = memo[(bits * 2654435761u) >> 18];
            if (e.key != bits + 1) {
                const double y0 = -(f + 3) * kPi * 0.25;
                e               = Entry{bits + 1, std::sin(y0), std::cos(y0)};
            }
            L.s0 = e.s, L.c0 = e.c;
        }
        out[d - d0] = L;
    }
}

// One resize_generic launch: its jobs, the Lanczos tap tables, and the tile shape every job of it
// shares (rows x columns of a tile sized so the taps and the horizontal sums fit 64 KiB of LDS).
struct GrPlan {
    std::vector<ResizeJob> jobs;
    size_t                 off = 0, lz_off = 0, taps_off = 0; // byte offsets in the call's table
    // One launch per method class (finalize sorts the jobs so each class is contiguous): the
    // fixed-K methods as resize_sep bands, the rest (INTER_AREA's float taps, integer boxes, jobs
    // whose bands do not fit) as resize_generic tiles.
    struct Sub {
        int  first = 0, count = 0;
        int  TR = 16, CW = 128, NR = 1, xs = 3, amax = 1, cn_max = 1, max_tiles = 0, SW = 4;
        int  sep = 0;           // K of resize_sep, or 0: resize_generic
        bool area = false;      // resize_sep's INTER_AREA form (resizeArea_ jobs, sep = their most taps)
        bool any_final = false; // some job writes the loader's output itself (its LUT in the launch's LDS)
    };
    std::vector<Sub> subs;
    double bytes = 0; // algorithmic: the source region read once + the window written

    size_t n_taps = 0;     // Lanczos4 taps reserved by add(), their inputs computed by fill_taps()
    size_t n_taps_max = 0; // ... and what the jobs would need with no axis shared (the ring's sizing bound)
    // One tap array per distinct axis (source size, scale, first destination index, count, column clamp):
    // a batch of random crops over one output size repeats them (C2: ~76 crop widths, ~76 heights for 512
    // axes of 256 records), and equal inputs give equal taps.
    struct LzAxis {
        int      ssize, d0, n, clamp;
        uint64_t scale_bits;
        bool     operator==(const LzAxis& o) const
        {
            return ssize == o.ssize && d0 == o.d0 && n == o.n && clamp == o.clamp && scale_bits == o.scale_bits;
        }
    };
    struct LzAxisHash {
        size_t operator()(const LzAxis& a) const
        {
            uint64_t h = a.scale_bits * 0x9E3779B97F4A7C15ull;
            for (int v : {a.ssize, a.d0, a.n, a.clamp}) h = (h ^ (uint32_t)v) * 0x100000001B3ull;
            return (size_t)h;
        }
    };
    std::unordered_map<LzAxis, size_t, LzAxisHash> lz_index; // axis -> its first tap
    std::vector<std::pair<LzAxis, size_t>>          lz_axes;  // (axis, first tap), in reservation order
    int32_t axis_taps(int ssize, double scale, int d0, int n, bool clamp)
    {
        LzAxis a{ssize, d0, n, clamp ? 1 : 0, 0};
        std::memcpy(&a.scale_bits, &scale, 8);
        auto it = lz_index.find(a);
        if (it == lz_index.end()) {
            it = lz_index.emplace(a, n_taps).first;
            lz_axes.emplace_back(a, n_taps);
            n_taps += n;
        }
        return (int32_t)(it->second * sizeof(GrTap));
    }

    void add(ResizeJob R)
    {
        if (R.method == GR_LANCZOS4) { // byte offsets, relative until the table is laid out
            n_taps_max += (size_t)R.win_w + R.win_h;
            R.coef_x = axis_taps(R.crop_w, R.scale_x, R.win_x, R.win_w, true);
            R.coef_y = axis_taps(R.crop_h, R.scale_y, R.win_y, R.win_h, false);
        }
        jobs.push_back(R);
    }
    // The Lanczos4 tap inputs (a sin and a cos per destination column and row), on `pool` when there
    // are enough jobs to pay for it; the device turns them into the taps (the whole taps computed here
    // cost ~75 us per 224x224 record of libm, divisions and rounding: ~1.1 ms per 256-record call on
    // 14 threads, and the LANCZOS4 step was host-bound).
    // They go straight into the call's pinned table (`lz`: n_taps entries; a per-call vector of ~2.8 MB
    // and its copy into the table cost page faults under 14 writers and ~0.1 ms of memcpy).
    void fill_taps(thread_pool* pool, LzIn* lz) const
    {
        auto one = [&](int i) {
            const LzAxis& a = lz_axes[i].first;
            double        scale;
            std::memcpy(&scale, &a.scale_bits, 8);
            lanczos4_inputs(a.ssize, scale, a.d0, a.n, a.clamp != 0, lz + lz_axes[i].second);
        };
        if (pool && n_taps > 4096) pool->run((int)lz_axes.size(), one);
        else for (int i = 0; i < (int)lz_axes.size(); i++) one(i);
    }
    static int ksize(int m) { return m == GR_CUBIC ? 4 : (m == GR_LANCZOS4 ? 8 : 2); }
    static int sep_k(int m) { return m == GR_CUBIC ? 4 : m == GR_LANCZOS4 ? 8 : m == GR_LINEAR_AREA ? 2 : 0; }
    // launch classes: the fixed-K methods by K, resizeArea_ jobs, the rest
    static int cls(int m) { return sep_k(m) ? sep_k(m) : m == GR_AREA ? 50 : 99; }
    // rows of H a tile of `tr` output rows needs at most (jobs [f, f + n))
    int rows_for(int f, int n, int tr) const
    {
        int nr = 1;
        for (int i = f; i < f + n; i++) {
            const ResizeJob& R = jobs[i];
            if (R.method == GR_AREA) nr = std::max(nr, (int)std::ceil(tr * R.scale_y) + 3);
            else if (R.method != GR_AREA_FAST) nr = std::max(nr, (int)std::ceil((tr - 1) * R.scale_y) + ksize(R.method) + 2);
        }
        return nr;
    }
    // staged source bytes per row a tile of `cw` output columns needs at most (a multiple of 4)
    int bytes_for(int f, int n, int cw) const
    {
        int sw = 4;
        for (int i = f; i < f + n; i++) {
            const ResizeJob& R = jobs[i];
            int              cols = 1;
            if (R.method == GR_AREA) cols = (int)std::ceil(cw * R.scale_x) + 4;
            else if (R.method != GR_AREA_FAST) cols = (int)std::ceil((cw - 1) * R.scale_x) + ksize(R.method) + 2;
            sw = std::max(sw, (std::min(cols, R.crop_w) * R.cn + 3) / 4 * 4);
        }
        return sw;
    }
    // the launch shape of jobs [f, f + n): resize_sep when they are one fixed-K class of one channel
    // count and a band fits, else resize_generic
    Sub shape(int f, int n) const
    {
        Sub u;
        u.first = f, u.count = n;
        for (int i = f; i < f + n; i++) u.any_final = u.any_final || jobs[i].final_out;
        const size_t lut_lds = u.any_final ? 768 * 4 : 0;
        int          K = 2, ww = 1;
        for (int i = f; i < f + n; i++) {
            const ResizeJob& R = jobs[i];
            K = std::max(K, ksize(R.method));
            if (R.method == GR_AREA) u.amax = std::max(u.amax, (int)std::ceil(std::max(R.scale_x, R.scale_y)) + 3);
            u.cn_max = std::max(u.cn_max, R.cn);
            ww       = std::max(ww, R.win_w);
        }
        // resize_sep: bands of up to 32 rows x the window's width (at most 256 lanes of 4 bytes); resizeArea_
        // jobs as its INTER_AREA form, K = their most taps per destination index (floor(scale) + 2)
        int               ka      = 0;
        static const bool no_area = std::getenv("AEON_HIP_AREA_SEP") && std::atoi(std::getenv("AEON_HIP_AREA_SEP")) == 0;
        if (jobs[f].method == GR_AREA && !no_area) { // (development: AEON_HIP_AREA_SEP=0, resize_generic)
            double smax = 1;
            for (int i = f; i < f + n; i++) smax = std::max({smax, jobs[i].scale_x, jobs[i].scale_y});
            const int taps = (int)std::floor(smax) + 2;
            ka             = taps <= 4 ? 4 : taps <= 8 ? 8 : 0;
        }
        const int sk  = ka ? ka : sep_k(jobs[f].method);
        const int xs  = (ka ? 2 : 1) + sk;
        bool      one = sk != 0;
        for (int i = f; i < f + n; i++) one = one && jobs[i].method == jobs[f].method && jobs[i].cn == u.cn_max;
        if (one) {
            static const int tr0 = std::getenv("AEON_HIP_SEP_TR") ? std::atoi(std::getenv("AEON_HIP_SEP_TR")) : 16;
            // a band's lanes (at most 256): 4 bytes of a u8 window row each, or 4 pixels of one channel of a
            // final_out job each -- cn * ceil(cw / 4) lanes, so 340 columns for 3 channels, not 341
            int cw = std::min({ww, 1024 / u.cn_max, 4 * (256 / u.cn_max)}), tr = std::max(4, std::min(64, tr0));
            // staged rows: whole 16-byte blocks (resize_sep), hence up to 30 bytes more per row, and 32
            // bytes of room for the replicated borders (resize_kernels.hip kSepPadL)
            auto sw = [&] { return (bytes_for(f, n, cw) + 30 + 15) / 16 * 16 + 32; };
            auto l  = [&] {
                return ((size_t)(cw + tr) * xs * 4 + 15) / 16 * 16 + (size_t)rows_for(f, n, tr) * sw() + lut_lds;
            };
            while (l() > kSepLds && tr > 4) tr /= 2;
            if (l() <= kSepLds) {
                u.sep = sk, u.area = ka != 0, u.TR = tr, u.CW = cw, u.NR = rows_for(f, n, tr), u.SW = sw(), u.xs = xs;
                return u;
            }
        }
        u.xs = std::max(1 + K, 2 + u.amax);
        u.CW = std::min(128, ww);
        u.TR = 16;
        // with the source rows staged in LDS (SW > 0) when they fit at 16 x 128 tiles, else without
        bool staged = true;
        auto lds    = [&] {
            return ((size_t)u.CW * u.xs + (size_t)u.TR * u.xs + (size_t)rows_for(f, n, u.TR) * u.CW * u.cn_max) * 4 +
                   (staged ? (size_t)rows_for(f, n, u.TR) * bytes_for(f, n, u.CW) : 0) + lut_lds;
        };
        staged = lds() <= kGenericLds;
        while (lds() > kGenericLds && u.TR > 1) u.TR--;
        while (lds() > kGenericLds && u.CW > 8) u.CW /= 2;
        if (lds() > kGenericLds) fail(AEON_HIP_EUNSUPPORTED, "resize scale too large for the generic resize's LDS tiles");
        u.NR = rows_for(f, n, u.TR);
        u.SW = staged ? bytes_for(f, n, u.CW) : 0;
        return u;
    }
    void finalize()
    {
        subs.clear();
        bytes = 0;
        if (jobs.empty()) return;
        // the classes contiguous: resize_sep's by K, resizeArea_'s, then the other generic methods
        std::stable_sort(jobs.begin(), jobs.end(), [](const ResizeJob& a, const ResizeJob& b) { return cls(a.method) < cls(b.method); });
        for (int f = 0; f < (int)jobs.size();) {
            int e = f + 1;
            while (e < (int)jobs.size() && cls(jobs[e].method) == cls(jobs[f].method)) e++;
            subs.push_back(shape(f, e - f));
            f = e;
        }
        for (Sub& u : subs) {
            u.max_tiles = 0;
            for (int i = u.first; i < u.first + u.count; i++) {
                ResizeJob& R = jobs[i];
                R.tiles_x    = (R.win_w + u.CW - 1) / u.CW;
                R.tiles      = R.tiles_x * ((R.win_h + u.TR - 1) / u.TR);
                u.max_tiles  = std::max(u.max_tiles, R.tiles);
                bytes += (double)R.crop_w * R.crop_h * R.cn * ((double)R.win_w / R.dst_w) * ((double)R.win_h / R.dst_h) +
                         (double)R.win_w * R.win_h * R.cn * (R.final_out ? 4 : 1);
            }
        }
    }
    static constexpr size_t kGenericLds = 64 * 1024;
    static constexpr size_t kSepLds     = 40 * 1024; // (four bands per CU)
};

// A resize of the (cropped, padded) region of J's source to its window, into scratch at `off`.
// (development: AEON_HIP_IDENTITY_SEP=0 keeps identity resizes on the tile kernel)
bool no_identity_sep()
{
    static const bool v = std::getenv("AEON_HIP_IDENTITY_SEP") && std::atoi(std::getenv("AEON_HIP_IDENTITY_SEP")) == 0;
    return v;
}

ResizeJob resize_job(const AugJob& J, int method, int isx, int isy)
{
    ResizeJob R{};
    R.scale_x = J.scale_x, R.scale_y = J.scale_y;
    R.inv_x = (double)J.dst_w / J.crop_w, R.inv_y = (double)J.dst_h / J.crop_h;
    R.src_ptr = J.src_ptr, R.src_scratch = J.src_scratch;
    R.src_stride = J.src_stride, R.cn = J.cn;
    R.crop_x = J.crop_x, R.crop_y = J.crop_y, R.crop_w = J.crop_w, R.crop_h = J.crop_h;
    R.shift_x = J.shift_x, R.shift_y = J.shift_y, R.padded = J.padded;
    R.dst_w = J.dst_w, R.dst_h = J.dst_h;
    R.win_x = J.win_x, R.win_y = J.win_y, R.win_w = J.win_w, R.win_h = J.win_h;
    R.method = method, R.isx = isx, R.isy = isy;
    return R;
}

// Launch order: rot (image::rotate) -> exp (image::expand) -> gr_short / pre (resize_short, generic
// or tile) -> gr_main (CUBIC / LANCZOS4 / AREA resize of the crop) -> pre2 (2x-area resize ahead of
// photometric stages) -> pass1 (contrast statistics) -> main; each reads only what an earlier group
// wrote.
void plan_image(const aeon_img_desc& d, const void* src_base, const aeon_aug_params& p,
                const aeon_out_desc& o, uint8_t* out_item, bool is_mask, std::vector<RotJob>& rot,
                std::vector<ExpandJob>& exp, GrPlan& gr_short, LaunchPlan& pre, GrPlan& gr_main, LaunchPlan& pre2,
                LaunchPlan& pass1, LaunchPlan& main, size_t& scratch_bytes)
{
    validate_record(d, p, o, is_mask);
    const int cn = d.channels;
    AugJob    J;
    plan_direct(d, (uint64_t)src_base, p, out_geom(o), (uint64_t)out_item, is_mask, J);
    if (p.angle != 0) {
        // image::rotate into scratch (interpolated for images, nearest + border 0 for pixel
        // masks, etl_pixel_mask.cpp:72-74); everything after reads the rotated record
        // Only the cropbox window is produced when nothing before the crop needs the whole rotated
        // record (no expand canvas, no resize_short of it); the job then crops it at (0, 0).
        RotJob R{};
        rotation_inverse_map(d.width, d.height, p.angle, R.M);
        R.src_ptr = J.src_ptr;
        R.w = d.width, R.h = d.height, R.stride = d.stride, R.cn = cn;
        R.interp = is_mask ? AEON_INTERP_NEAREST : AEON_INTERP_LINEAR;
        const bool window = is_mask || (!expands(p) && p.resize_short_size <= 0);
        R.ox = window ? p.crop_x : 0, R.oy = window ? p.crop_y : 0;
        R.ow = window ? p.crop_w : d.width, R.oh = window ? p.crop_h : d.height;
        size_t off    = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)R.ow * R.oh * cn + 16;
        R.out_ptr     = off; // relocated to the slot's scratch by the caller
        R.angle       = p.angle;
        rot.push_back(R);
        J.src_ptr     = off;
        J.src_scratch = 1;
        J.src_w = R.ow, J.src_h = R.oh;
        J.src_bytes   = (uint64_t)R.ow * R.oh * cn;
        J.src_stride  = R.ow * cn;
        J.crop_x -= R.ox, J.crop_y -= R.oy;
    }
    if (!is_mask && expands(p)) {
        // image::expand (image.cpp:276-303) into scratch: a zeroed expand_w x expand_h canvas with the
        // (rotated) record at (expand_x, expand_y); everything after reads the canvas
        ExpandJob E{};
        E.src_ptr     = J.src_ptr;
        E.src_scratch = J.src_scratch;
        E.w = J.src_w, E.h = J.src_h, E.stride = J.src_stride, E.cn = cn;
        E.ew = p.expand_w, E.eh = p.expand_h, E.ox = p.expand_x, E.oy = p.expand_y;
        size_t off    = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)E.ew * E.eh * cn + 16;
        E.out_ptr     = off; // relocated to the slot's scratch by the caller
        exp.push_back(E);
        J.src_ptr     = off;
        J.src_scratch = 1;
        J.src_bytes   = (uint64_t)E.ew * E.eh * cn;
        J.src_w = E.ew, J.src_h = E.eh, J.src_stride = E.ew * cn;
    }
    if (!is_mask && p.resize_short_size > 0) {
        // image::resize_short (image.cpp:118-127) into a device scratch, cropbox window only
        const int bw = J.src_w, bh = J.src_h; // the (rotated, expanded) record
        int       rw, rh;
        get_resized_short_size(bw, bh, p.resize_short_size, &rw, &rh);
        AugJob P = J;
        P.photo   = 0;
        P.flip    = 0;
        P.shift_x = P.shift_y = P.padded = 0;
        P.crop_x = 0, P.crop_y = 0, P.crop_w = bw, P.crop_h = bh;
        P.mode    = choose_mode(bw, bh, rw, rh, p.interp, cn);
        P.scale_x = 1. / ((double)rw / bw);
        P.scale_y = 1. / ((double)rh / bh);
        P.dst_w = rw, P.dst_h = rh;
        P.win_x = p.crop_x, P.win_y = p.crop_y, P.win_w = p.crop_w, P.win_h = p.crop_h;
        P.xv      = simd_boundary(rw * cn);
        size_t off = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)p.crop_w * p.crop_h * cn + 16;
        P.out_ptr = off; // relocated to the slot's scratch by the caller
        int       isx = 0, isy = 0;
        const int gm  = generic_method(bw, bh, rw, rh, p.interp, cn, &isx, &isy);
        if (gm >= 0) {
            ResizeJob R   = resize_job(P, gm, isx, isy);
            R.out_ptr     = off;
            R.out_scratch = 1;
            gr_short.add(R);
        } else {
            pre.jobs.push_back(P);
        }
        J.src_ptr = off; // likewise
        J.src_bytes  = (uint64_t)p.crop_w * p.crop_h * cn;
        J.src_w = p.crop_w, J.src_h = p.crop_h, J.src_stride = p.crop_w * cn;
        J.crop_x = 0, J.crop_y = 0;
        J.src_scratch = 1; // relocated to the slot's scratch by the caller
    }
    int       isx = 0, isy = 0;
    int       gm  = is_mask ? -1 : generic_method(J.crop_w, J.crop_h, J.dst_w, J.dst_h, p.interp, cn, &isx, &isy);
    const bool final_ok = J.photo == 0 && o.dtype == AEON_DTYPE_F32 && !o.fixed_aspect_ratio && (cn == 1 || cn == 3) &&
                          o.channels == cn;
    // An identity resize (cv::resize copies) of a CUBIC / LANCZOS4 / INTER_AREA call with no photometric
    // stage and f32 output: through the call's resize class with identity taps -- (0, 2048, 0, 0), the
    // fraction-0 Lanczos row, the bilinear emulation's (2048, 0), each reproducing the byte exactly -- so
    // the call launches no tile kernel for its few uncropped records (an 8.5 us launch per C2:<method>
    // step: one tile's latency).
    if (gm < 0 && !is_mask && final_ok && J.crop_w == J.dst_w && J.crop_h == J.dst_h &&
        (p.interp == AEON_INTERP_CUBIC || p.interp == AEON_INTERP_LANCZOS4 || p.interp == AEON_INTERP_AREA) && !no_identity_sep())
        gm = p.interp == AEON_INTERP_CUBIC ? GR_CUBIC : p.interp == AEON_INTERP_LANCZOS4 ? GR_LANCZOS4 : GR_LINEAR_AREA;
    if (gm >= 0 && gm != GR_AREA_FAST && final_ok) {
        // no photometric stage and f32 output: the resize pass is the last one -- it flips,
        // standardizes through the LUT and stores the loader's layout itself (no u8 window in scratch,
        // no copy pass)
        ResizeJob R = resize_job(J, gm, isx, isy);
        R.out_ptr   = J.out_ptr;
        R.final_out = 1, R.flip = J.flip, R.out_pitch = J.out_pitch, R.out_plane = J.out_plane;
        gr_main.add(R);
        return;
    }
    if (gm >= 0) {
        // CUBIC / LANCZOS4 / INTER_AREA resize of the (padded) crop into scratch (resize_kernels.hip),
        // then the photometric stages, flip and the loader as a copy pass over it
        ResizeJob R   = resize_job(J, gm, isx, isy);
        size_t    off = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)J.win_w * J.win_h * cn + 16;
        R.out_ptr     = off; // relocated to the slot's scratch by the caller
        R.out_scratch = 1;
        gr_main.add(R);
        J.src_ptr     = off;
        J.src_scratch = 1;
        J.src_bytes   = (uint64_t)J.win_w * J.win_h * cn;
        J.src_w = J.win_w, J.src_h = J.win_h, J.src_stride = J.win_w * cn;
        J.crop_x = J.crop_y = 0, J.crop_w = J.win_w, J.crop_h = J.win_h;
        J.shift_x = J.shift_y = J.padded = 0;
        J.mode    = RESIZE_COPY;
        J.scale_x = J.scale_y = 1.0;
        J.xv      = simd_boundary(J.win_w * cn);
    }
    const int photo = J.photo;
    if (photo && J.mode == RESIZE_AREA2X) {
        // 2x-area resize first (resize-only pre-pass into scratch, unflipped), then the
        // photometric stages as a copy pass over it
        AugJob P      = J;
        P.photo       = 0;
        P.flip        = 0;
        size_t off    = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)J.win_w * J.win_h * 3 + 16;
        P.out_ptr     = off; // relocated to the slot's scratch by the caller
        pre2.jobs.push_back(P);
        J.src_ptr     = off;
        J.src_scratch = 1;
        J.src_bytes   = (uint64_t)J.win_w * J.win_h * 3;
        J.src_w = J.win_w, J.src_h = J.win_h, J.src_stride = J.win_w * 3;
        J.crop_x = J.crop_y = 0, J.crop_w = J.win_w, J.crop_h = J.win_h;
        J.shift_x = J.shift_y = J.padded = 0;
        J.mode    = RESIZE_COPY;
        J.scale_x = J.scale_y = 1.0;
        J.xv      = simd_boundary(J.win_w * 3);
    }
    if (photo & PHOTO_CONTRAST) {
        // contrast needs the mean of the post-hue image: pass 1 writes that image (HWC
        // uint8, unflipped) and its exact per-chunk sums; pass 2 (this job) reads it back
        AugJob P1     = J;
        P1.flip       = 0;
        P1.photo      = photo & (PHOTO_BS | PHOTO_HUE | PHOTO_CONTRAST);
        P1.stats_slot = (int)pass1.jobs.size();
        size_t off    = (scratch_bytes + 15) & ~(size_t)15;
        scratch_bytes = off + (size_t)J.win_w * J.win_h * 3 + 16;
        P1.out_ptr    = off; // relocated to the slot's scratch by the caller
        pass1.jobs.push_back(P1);
        J.stats_slot  = P1.stats_slot;
        J.src_ptr     = off;
        J.src_scratch = 1;
        J.src_bytes   = (uint64_t)J.win_w * J.win_h * 3;
        J.src_w = J.win_w, J.src_h = J.win_h, J.src_stride = J.win_w * 3;
        J.crop_x = J.crop_y = 0, J.crop_w = J.win_w, J.crop_h = J.win_h;
        J.shift_x = J.shift_y = J.padded = 0;
        J.mode    = RESIZE_COPY;
        J.scale_x = J.scale_y = 1.0;
        J.xv      = simd_boundary(J.win_w * 3);
        J.photo   = photo & (PHOTO_CONTRAST | PHOTO_LIGHTING);
    }
    if ((J.out_ptr & 15) != 0 || (J.win_w & 3) != 0 || o.fixed_aspect_ratio) main.vec_ok = false;
    main.jobs.push_back(J);
}

// ---------------------------------------------------------------------------------------------
// Context: per-GPU state and a 4-deep staging ring (pinned host blob -> device blob per call)
// ---------------------------------------------------------------------------------------------
struct Slot {
    hipEvent_t done     = nullptr; // the slot's kernels finished (host reuses the slot after it)
    hipEvent_t copied   = nullptr; // the slot's job table reached the device
    bool       pending  = false; // the slot's kernels may still run: wait for slots[cover].done
    int        cover    = -1;
    uint8_t*   host     = nullptr;
    size_t     host_cap = 0;
    uint8_t*   host_dev = nullptr; // device view of `host` (zero-copy job tables)
    uint8_t*   dev      = nullptr;
    size_t     dev_cap  = 0;
    uint8_t*   vram     = nullptr; // job tables the host writes straight into HBM (uncached, through the BAR)
    size_t     vram_cap = 0;
    uint8_t*   scratch  = nullptr;
    size_t     scratch_cap = 0;
    uint32_t*  partials = nullptr;
    size_t     partials_cap = 0;
    double*    shifts = nullptr; // contrast (1-c)*mean per stats slot (contrast_reduce)
    size_t     shifts_cap = 0;
};

} // namespace

constexpr int kTimerJpeg = 3; // KernelTimer kind of the JPEG kernels (after the KernelMode kinds)
struct KernelTimer {
    hipEvent_t start, stop;
    int        kind;   // KernelMode, or kTimerJpeg
    double     bytes;  // algorithmic bytes of the launch
};

struct aeon_hip_ctx {
    int        device = 0;
    int32_t*   d_error = nullptr; // kErrWords device error words: [0] the null stream's (and overflow),
                                  // [i] the i-th stream's (stream_error)
    static constexpr int kErrWords = 64;
    hipStream_t err_stream[kErrWords] = {};
    std::mutex  err_mu;
    int32_t*    call_error = nullptr; // the word of the call in progress (run_batch, under mu)
    uint32_t*  d_tail  = nullptr; // per ring slot: dynamic-tail tile counters (zero between launches)
    int32_t*   d_hsv   = nullptr;
    // staging ring: a slot (job table, scratch) is reused only after the kernels that read it
    // finished.  A completion event is recorded once per `done_every` calls on a stream and
    // covers the calls since the previous one (each event costs GPU time between launches).
    static constexpr int kSlots = 16;
    Slot       slots[kSlots];
    int        next = 0;
    int        done_every = 8;
    size_t     table_cap = 0, partials_cap = 0, shifts_cap = 0; // per-slot capacities (ensure_ring)
    // direct calls (run_direct): records of one job each, one launch group: the tile kernel reads
    // the jobs from the pinned slot itself
    bool                 direct = true; // AEON_HIP_DIRECT=0: the multi-pass path (device job table) for every call
    bool                 records = true; // AEON_HIP_RECORDS=0: contrast calls through the two-launch path
    int                  rec_helpers = 2; // AEON_HIP_REC_HELPERS: staging-only waves of the record kernel
    int                  rec_phases  = 0; // AEON_HIP_REC_PHASES (development): row phases of the record kernel
    bool                 split = false;     // AEON_HIP_SPLIT=1: non-photometric INTER_LINEAR f32 launches through
                                            // augment_split (measured slower than augment_tiles)
    int                  split_helpers = 2; // AEON_HIP_SPLIT_HELPERS: staging waves of augment_split
    int                  split_rpl = 2;     // AEON_HIP_SPLIT_RPL: output rows per compute lane per tile
    int                  split_occ = 1;     // AEON_HIP_SPLIT_OCC: augment_split workgroups per CU (1 or 2)
    bool                 fuse_masks = false; // AEON_HIP_FUSE_MASKS=1: a pair call's masks inside the image launch
    bool                 vram_jobs = false; // job tables written by the host into device memory (large-BAR GPUs;
                                            // AEON_HIP_VRAM_JOBS=0: pinned host tables)
    bool                 jpeg_gpu_huff = true; // AEON_HIP_JPEG_HUFF=host: every JPEG through the host entropy decoder
    std::vector<JobGeom> geoms;              // reused per call
    std::vector<AugJob>  direct_jobs;        // (run_direct) the call's jobs before they go into the slot
    std::vector<int>     direct_order;       // (run_direct) their table order: largest crop first
    JpegState*           jpeg = nullptr;     // JPEG decode stage (pool, staging ring), on first use
    thread_pool*         host_pool = nullptr; // the owning decoder's pool (ctx_share_pool), for the JPEG stage
    std::unique_ptr<thread_pool> plan_pool;        // the context's own, made for the first call with many Lanczos4 taps
    std::vector<int> open_slots; // used since the last completion event, on open_stream
    hipStream_t      open_stream = nullptr;
    // job tables go up on their own stream, so a call's H2D overlaps the previous call's kernels
    // instead of queueing between them on the caller's stream
    hipStream_t copy_stream = nullptr;
    int         n_cu      = 0;
    std::vector<std::pair<std::vector<int>, int>> occ; // launch shape -> workgroups per CU
    // standardize LUTs stay resident per distinct output config (a new one is uploaded once)
    struct Lut {
        float  host[768];
        float* dev = nullptr;
    };
    std::vector<Lut> luts;
    aeon_out_desc    lut_memo_od{}; // the last resident_lut call: its config and LUT
    bool             lut_memo_u8  = false;
    const float*     lut_memo_dev = nullptr;
    // per-launch timing events on every `timing_every`-th call only (they cost GPU time)
    int         timing_every = 1;
    long        timing_calls = 0;
    std::mutex mu;
    // optional per-launch timing (aeon_hip_set_timing): events recorded on the launch stream
    bool                     timing = false;
    std::vector<KernelTimer> timers, free_timers;
    double                   ms[4]    = {0, 0, 0, 0};
    // AEON_HIP_HOST_PROFILE=1: host time per run_batch phase, printed when the context is destroyed
    bool                     host_profile = false;
    std::vector<double>      host_ns[8];  // per call, per phase
    long                     host_calls   = 0;
    double                   bytes[4] = {0, 0, 0, 0};
    long                     count[4] = {0, 0, 0, 0};
#ifdef AEON_HIP_TRACE
    uint32_t*                trace = nullptr; // AEON_HIP_TRACE_PTR, read once at ctx_create
#endif
};

struct aeon_param_factory {
    param_factory f;
    std::mutex    mu; // make_params calls are serialised (the lighting normal_distribution caches a draw)
    explicit aeon_param_factory(const Json& j) : f(j) {}
};

namespace {

void grow(uint8_t*& p, size_t& cap, size_t need, bool pinned)
{
    if (need <= cap) return;
    size_t n = std::max(need, cap * 2);
    if (p) HIP_OK(pinned ? hipHostFree(p) : hipFree(p));
    p   = nullptr;
    cap = 0;
    if (pinned) HIP_OK(hipHostMalloc((void**)&p, n, hipHostMallocDefault));
    else HIP_OK(hipMalloc((void**)&p, n));
    cap = n;
}

void close_slots(aeon_hip_ctx* ctx);

// Device memory the host writes directly (a large-BAR GPU maps all of it): uncached, so every GPU read
// of it -- a kernel's job fetch -- goes to HBM and never meets a stale cache line of the slot's
// previous call.
// The host may write through p when the page holding it is mapped read-write into this process (on a
// large-BAR GPU the driver maps host-visible VRAM at the allocation's own address; a restricted or
// virtualised BAR can allocate device memory without mapping it for the CPU, and the runtime reports no
// host pointer for device memory either way).  Checked in /proc/self/maps -- no signal handlers, nothing
// process-wide touched, safe next to other threads -- then one write + read-back through p.
bool host_mapped_rw(const void* p, size_t bytes)
{
    std::FILE* f = std::fopen("/proc/self/maps", "r");
    if (!f) return false;
    const unsigned long a  = (unsigned long)(uintptr_t)p;
    bool                ok = false;
    char                line[512];
    while (std::fgets(line, sizeof line, f)) {
        unsigned long lo = 0, hi = 0;
        char          perms[8] = {0};
        if (std::sscanf(line, "%lx-%lx %7s", &lo, &hi, perms) != 3) continue;
        if (a >= lo && a < hi) {
            ok = a + bytes <= hi && perms[0] == 'r' && perms[1] == 'w';
            break;
        }
    }
    std::fclose(f);
    return ok;
}
bool host_can_write(void* p)
{
    if (!host_mapped_rw(p, sizeof(uint32_t))) return false;
    volatile uint32_t* q = (volatile uint32_t*)p;
    q[0]                 = 0xA5C3E1F7u;
    return q[0] == 0xA5C3E1F7u;
}

// The uncached HBM tables are never handed back to the driver: a context's tables go into a process-wide
// pool when it is destroyed (or grows them) and the next context takes them from there.  Measured on the
// MI355X boxes: once an uncached block had been freed, a later ordinary device allocation that reused its
// memory lost writes -- 128-byte lines of a kernel's output read back as zeros by the next kernel on the
// stream (tests/test_decoder.py after the stager and JPEG tests: 1-2.7 KB of one record, in 3 of 3
// runs; with the pool, 0 of 2; with cached tables, or pinned ones, 0 of 4).
std::mutex                               g_vram_pool_mu;
std::vector<std::pair<uint8_t*, size_t>> g_vram_pool;   // released tables, still allocated and mapped
std::vector<uint8_t*>                    g_vram_unused; // blocks whose probe failed (kept, never used)
std::vector<std::pair<uint8_t*, size_t>> g_vram_all;    // every uncached block of the process (diagnostics)
void free_vram(uint8_t*& p, size_t& cap)
{
    if (p) {
        std::lock_guard<std::mutex> lock(g_vram_pool_mu);
        g_vram_pool.emplace_back(p, cap);
    }
    p = nullptr, cap = 0;
}

bool grow_vram(int device, uint8_t*& p, size_t& cap, size_t need) // false: no table (p released)
{
    if (need <= cap) return true;
    const size_t n = std::max(need, cap * 2);
    free_vram(p, cap);
    {
        std::lock_guard<std::mutex> lock(g_vram_pool_mu); // the smallest pooled block of this device that fits
        size_t best = g_vram_pool.size();
        for (size_t i = 0; i < g_vram_pool.size(); i++) {
            hipPointerAttribute_t at{};
            if (g_vram_pool[i].second < n || hipPointerGetAttributes(&at, g_vram_pool[i].first) != hipSuccess ||
                at.device != device)
                continue;
            if (best == g_vram_pool.size() || g_vram_pool[i].second < g_vram_pool[best].second) best = i;
        }
        (void)hipGetLastError();
        if (best < g_vram_pool.size()) {
            p = g_vram_pool[best].first, cap = g_vram_pool[best].second;
            g_vram_pool.erase(g_vram_pool.begin() + (long)best);
            return true;
        }
    }
    if (hipExtMallocWithFlags((void**)&p, n, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        return false;
    }
    {
        std::lock_guard<std::mutex> lock(g_vram_pool_mu);
        g_vram_all.emplace_back(p, n);
    }
    // the host writes these tables through p itself: only when p's page is mapped read-write for the
    // host and a write + read-back through p works (a restricted BAR or a virtualised GPU can allocate it without mapping it for the
    // CPU; the runtime reports no host pointer for device memory either way) -- the pinned paths then
    if (!host_can_write(p)) {
        (void)hipGetLastError();
        if (std::getenv("AEON_HIP_HOST_PROFILE"))
            std::fprintf(stderr, "[aeon_hip] uncached HBM block not host-writable: pinned job tables\n");
        std::lock_guard<std::mutex> lock(g_vram_pool_mu);
        g_vram_unused.push_back(p); // (not freed either: see above)
        p = nullptr;
        return false;
    }
    cap = n;
    return true;
}

// A call's job table (written in the slot's pinned `host` buffer) published where its kernels read it
// with device-memory latency: copied by the host into the slot's HBM table through the PCIe BAR
// (write-combined: one contiguous copy, then a full fence so the writes reach the device ahead of the
// launch's doorbell).  Null when the context has no such tables.  (C2: the workgroups' first job
// fetch waited 3.7 us over PCIe from pinned memory, 0.3 us from HBM; tools/trace_kernel.py.)
constexpr size_t kVramTableMax = 1 << 20;
const uint8_t* publish_table(aeon_hip_ctx* ctx, Slot& s, size_t bytes)
{
    if (!ctx->vram_jobs || bytes == 0 || bytes > kVramTableMax || bytes > s.vram_cap) return nullptr;
    std::memcpy(s.vram, s.host, bytes);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    // a read back through the BAR: PCIe does not let a read pass the posted writes ahead of it, so
    // the table is in HBM when it returns (~1 us of host time; the host runs ahead of the GPU)
    (void)*(volatile const uint32_t*)(s.vram + ((bytes - 1) & ~(size_t)3));
    return s.vram;
}

// publish_table for a table the host wrote into s.vram itself: the fence and the read-back only.
const uint8_t* publish_written(Slot& s, size_t bytes)
{
    std::atomic_thread_fence(std::memory_order_seq_cst);
    (void)*(volatile const uint32_t*)(s.vram + ((bytes - 1) & ~(size_t)3));
    return s.vram;
}

// Wait until no kernel of any ring slot can still be running.
void drain_ring(aeon_hip_ctx* ctx)
{
    close_slots(ctx);
    for (Slot& q : ctx->slots)
        if (q.pending) {
            HIP_OK(hipEventSynchronize(ctx->slots[q.cover].done));
            q.pending = false;
        }
}

// Ring capacities are shared by all slots and grown for all of them at once (after draining the
// ring), so the first call -- a warmup -- allocates everything the steady state needs and later
// calls never pay an allocation when they rotate onto a slot they have not used before.
void ensure_ring(aeon_hip_ctx* ctx, size_t table, size_t partials, size_t shifts)
{
    table = std::max<size_t>(table, 16);
    if (table <= ctx->table_cap && partials <= ctx->partials_cap && shifts <= ctx->shifts_cap) return;
    drain_ring(ctx);
    // (a quarter over the first need: a call's tables vary with its records' crops, and a later call
    // needing a few bytes more would otherwise reallocate every slot inside a loader's steady state --
    // ~10-20 ms of pinned and device allocations, seen as one-off stalls of the LANCZOS4 step)
    const size_t tc = table > ctx->table_cap ? std::max(table + table / 4, ctx->table_cap * 2) : ctx->table_cap;
    const size_t pc = partials > ctx->partials_cap ? std::max(partials + partials / 4, ctx->partials_cap * 2) : ctx->partials_cap;
    const size_t sc = shifts > ctx->shifts_cap ? std::max(shifts + shifts / 4, ctx->shifts_cap * 2) : ctx->shifts_cap;
    for (Slot& q : ctx->slots) {
        grow(q.host, q.host_cap, tc, true);
        HIP_OK(hipHostGetDevicePointer((void**)&q.host_dev, q.host, 0));
        grow(q.dev, q.dev_cap, tc, false);
        if (ctx->vram_jobs && !grow_vram(ctx->device, q.vram, q.vram_cap, std::min(tc, kVramTableMax))) {
            ctx->vram_jobs = false; // (no HBM tables on this device: the pinned paths)
            for (Slot& v : ctx->slots)
                free_vram(v.vram, v.vram_cap);
        }
        uint8_t* p = (uint8_t*)q.partials;
        grow(p, q.partials_cap, pc, false);
        q.partials = (uint32_t*)p;
        uint8_t* r = (uint8_t*)q.shifts;
        grow(r, q.shifts_cap, sc, false);
        q.shifts = (double*)r;
    }
    ctx->table_cap = tc, ctx->partials_cap = pc, ctx->shifts_cap = sc;
}

// Device copy of the standardize LUT of output config `o` (uploaded the first time it is seen).
const float* resident_lut(aeon_hip_ctx* ctx, const aeon_out_desc& o, bool u8_map = false)
{
    // the last call's output config again (a loader's steady state): its LUT without rebuilding it
    if (ctx->lut_memo_dev && ctx->lut_memo_u8 == u8_map && std::memcmp(&ctx->lut_memo_od, &o, sizeof(o)) == 0)
        return ctx->lut_memo_dev;
    float lut[768];
    build_lut(o, lut, u8_map);
    const float* dev = nullptr;
    for (auto& L : ctx->luts)
        if (std::memcmp(L.host, lut, sizeof(lut)) == 0) dev = L.dev;
    if (!dev) {
        if (ctx->luts.size() >= 16) { // many configs on one context: start over once the device is idle
            HIP_OK(hipDeviceSynchronize());
            for (auto& L : ctx->luts) HIP_OK(hipFree(L.dev));
            ctx->luts.clear();
        }
        aeon_hip_ctx::Lut L;
        std::memcpy(L.host, lut, sizeof(lut));
        HIP_OK(hipMalloc((void**)&L.dev, sizeof(lut)));
        HIP_OK(hipMemcpy(L.dev, lut, sizeof(lut), hipMemcpyHostToDevice));
        ctx->luts.push_back(L);
        dev = L.dev;
    }
    ctx->lut_memo_od  = o;
    ctx->lut_memo_u8  = u8_map;
    ctx->lut_memo_dev = dev;
    return dev;
}

// Algorithmic bytes of one launch: the resampled u8 source footprint plus
// the bytes written (KM_STATS / KM_RAW write an HWC uint8 intermediate).
template <typename J_>
double launch_bytes(const std::vector<J_>& jobs, int mode, size_t out_elem)
{
    double b = 0;
    for (const J_& J : jobs) {
        double rd = (double)J.crop_w * J.crop_h * J.cn;
        if (J.mode == RESIZE_LINEAR || J.mode == RESIZE_NEAREST) {
            // a window of the resize target reads only its share of the source
            rd *= ((double)J.win_w / J.dst_w) * ((double)J.win_h / J.dst_h);
        }
        double wr = (double)J.win_w * J.win_h * J.cn * (mode == KM_FINAL ? out_elem : 1);
        b += rd + wr;
    }
    return b;
}

// Persistent grid: as many workgroups as the CUs hold at once, never more than the tiles.
int grid_for(aeon_hip_ctx* ctx, int mode, const LaunchPlan& P, const LaunchArgs& a)
{
    int per_cu = 0;
    {
        const std::vector<int> key = {mode, P.rm, (int)P.tail, (int)P.photo, a.threads, a.lds_bytes, a.vec_ok, a.has_rtab,
                                      a.out_dtype, a.channel_major, a.m_blocks > 0};
        for (auto& e : ctx->occ)
            if (e.first == key) per_cu = e.second;
        if (per_cu <= 0) {
            HIP_OK(kernel_occupancy(mode, P.rm, P.tail, P.photo, a, &per_cu));
            per_cu = std::max(per_cu, 1);
            ctx->occ.push_back({key, per_cu});
            if (ctx->host_profile)
                std::fprintf(stderr, "[aeon_hip] kernel km=%d rm=%d tail=%d photo=%d: %d threads, %d B LDS, TR %d, "
                                     "%d workgroups/CU x %d CUs, %d tiles\n",
                             mode, P.rm, (int)P.tail, (int)P.photo, a.threads, a.lds_bytes, a.rows_per_tile, per_cu,
                             ctx->n_cu, a.total_tiles);
        }
    }
    return (int)std::min<long>((long)a.total_tiles, (long)per_cu * ctx->n_cu);
}

// One completion event after the open slots' kernels (on their stream) covers all of them.
void close_slots(aeon_hip_ctx* ctx)
{
    if (ctx->open_slots.empty()) return;
    const int last = ctx->open_slots.back();
    HIP_OK(hipEventRecord(ctx->slots[last].done, ctx->open_stream));
    for (int i : ctx->open_slots) ctx->slots[i].pending = true, ctx->slots[i].cover = last;
    ctx->open_slots.clear();
}

KernelTimer take_timer(aeon_hip_ctx* ctx, int kind, double bytes)
{
    KernelTimer t{};
    if (!ctx->free_timers.empty()) {
        t = ctx->free_timers.back();
        ctx->free_timers.pop_back();
    } else {
        // timing only: no system-scope fence (cache writeback + invalidate) when they complete,
        // which cost the stream ~11 us of idle GPU per timed launch
        HIP_OK(hipEventCreateWithFlags(&t.start, hipEventDisableSystemFence));
        HIP_OK(hipEventCreateWithFlags(&t.stop, hipEventDisableSystemFence));
    }
    t.kind  = kind;
    t.bytes = bytes;
    return t;
}

void timed_launch(aeon_hip_ctx* ctx, int mode, const LaunchPlan& P, const LaunchArgs& a, hipStream_t stream,
                  double bytes, bool timed)
{
    KernelTimer t{};
    if (timed) t = take_timer(ctx, mode, bytes);
    const int grid = grid_for(ctx, mode, P, a);
    HIP_OK(launch_tiles(mode, P.rm, P.tail, P.photo, a, grid, stream, timed ? t.start : nullptr,
                        timed ? t.stop : nullptr));
    if (timed) ctx->timers.push_back(t);
}

// The next ring slot for a call on `stream`, once the kernels that last used it are done.
Slot& take_slot(aeon_hip_ctx* ctx, hipStream_t stream, int& index)
{
    // calls on another stream than the open ones: close those with an event on their stream
    if (!ctx->open_slots.empty() && ctx->open_stream != stream) close_slots(ctx);
    index     = ctx->next;
    Slot& s   = ctx->slots[index];
    ctx->next = (ctx->next + 1) % aeon_hip_ctx::kSlots;
    if (s.pending) {
        HIP_OK(hipEventSynchronize(ctx->slots[s.cover].done));
        s.pending = false;
    }
    return s;
}

// The call's launches are enqueued: its slot stays busy until a completion event covers it.
void release_slot(aeon_hip_ctx* ctx, int index, hipStream_t stream)
{
    ctx->open_slots.push_back(index);
    ctx->open_stream = stream;
    if ((int)ctx->open_slots.size() >= ctx->done_every) close_slots(ctx);
    ctx->host_calls++;
}

// The loader side of a launch: ko = what the kernels write (fixed_aspect_ratio writes its uint8
// canvas whatever the declared type, u8_map = standardized through the LUT); double output
// standardizes in the kernel with the declared mean / stddev by source channel.
struct OutView {
    aeon_out_desc ko;
    bool          u8_map = false;
};
OutView out_view(const aeon_out_desc& o)
{
    OutView v;
    v.ko = o;
    if (o.fixed_aspect_ratio && o.dtype != AEON_DTYPE_U8) {
        v.ko.dtype    = AEON_DTYPE_U8;
        v.ko.has_mean = 0;
        v.u8_map      = o.has_mean != 0;
    }
    return v;
}

// The device error word of the calls on `stream`: each stream its own (so that aeon_hip_synchronize of
// one stream -- a decode window -- never reads or clears a bit another stream's kernels set meanwhile),
// the null stream and streams beyond the table's size share word 0.  A stream keeps its word until
// aeon_hip_synchronize has read it.
int32_t* stream_error(aeon_hip_ctx* ctx, hipStream_t stream, bool release = false)
{
    if (!stream) return ctx->d_error;
    std::lock_guard<std::mutex> lock(ctx->err_mu);
    int free_i = 0;
    for (int i = 1; i < aeon_hip_ctx::kErrWords; i++) {
        if (ctx->err_stream[i] == stream) {
            if (release) ctx->err_stream[i] = nullptr;
            return ctx->d_error + i;
        }
        if (!free_i && !ctx->err_stream[i]) free_i = i;
    }
    if (release || !free_i) return ctx->d_error;
    ctx->err_stream[free_i] = stream;
    return ctx->d_error + free_i;
}

LaunchArgs launch_args(aeon_hip_ctx* ctx, const Slot& s, const uint8_t* table, const LaunchPlan& L, int n_jobs,
                       const aeon_out_desc& o, const float* d_lut, int partial_stride, bool u8_map = false)
{
    LaunchArgs a{};
    // dynamic tail: the partial last round plus two full rounds before it drawn from a counter (one
    // or four full rounds measured within noise or slower), the slot's own counter so
    // launches of calls in flight never share one
    a.tail_ctr    = ctx->d_tail + (&s - ctx->slots);
#ifndef AEON_HIP_TAIL_ROUNDS
#define AEON_HIP_TAIL_ROUNDS 2
#endif
    a.tail_rounds = AEON_HIP_TAIL_ROUNDS;
    a.jobs           = (const AugJob*)(table + L.blob_off);
    a.job_bytes      = L.photo ? (int)sizeof(AugJob) : kJobHotBytes;
    a.job_stride     = (int)sizeof(AugJob);
    a.lut            = d_lut; // [3][256]: standardized, or (float)x without mean
    a.hsv_tables     = ctx->d_hsv;
    a.partials       = s.partials;
    a.shifts         = s.shifts;
    a.partial_stride = partial_stride;
    a.error          = ctx->call_error;
#ifdef AEON_HIP_TRACE
    a.trace = ctx->trace; // development builds only (tools/build_variants.sh trace)
#endif
    a.rows_per_tile = L.tr;
    a.max_tiles     = L.max_tiles;
    a.total_tiles   = L.max_tiles * n_jobs;
    a.stage_bytes   = L.stage_bytes;
    a.max_win_w     = L.max_win_w;
    a.out_dtype     = o.dtype;
    a.u8_map        = u8_map;
    a.has_mean      = o.has_mean;
    for (int c = 0; c < 3; c++) { // by source channel (mixChannels from_to {0,2,1,1,2,0} with bgr_to_rgb)
        const int oc = (o.bgr_to_rgb && o.channels == 3) ? 2 - c : c;
        a.smean[c]   = oc < o.channels ? o.mean[oc] : 0;
        a.sinv[c]    = oc < o.channels && o.stddev[oc] != 0 ? 1. / o.stddev[oc] : 0;
    }
    a.channel_major = o.channel_major;
    a.bgr_to_rgb    = o.bgr_to_rgb;
    a.vec_ok        = L.vec_ok && o.channel_major;
    a.lds_bytes     = L.lds;
    a.has_hue       = L.has_hue;
    a.threads       = L.threads;
    a.has_rtab      = L.rtab;
    return a;
}

// augment_split's shape for a direct call's records (all 3-channel, INTER_LINEAR, one window width W,
// W % 4 == 0): nwc compute waves of nph row phases x W/4 column groups plus ctx->split_helpers staging
// waves in one workgroup of <= 1,024 lanes, rows_per_tile = nph * rpl, two staging buffers.  The LDS
// request is held above half a CU's 160 KB so that the grid's n_cu workgroups land one per CU.  False:
// no such shape (the caller keeps augment_tiles).
template <typename J_>
bool plan_split(const aeon_hip_ctx* ctx, const std::vector<J_>& geo, LaunchPlan& P, SplitArgs& sa)
{
    if (geo.empty()) return false;
    const int W = geo[0].win_w;
    if (W <= 0 || (W & 3) != 0) return false;
    for (const J_& g : geo)
        if (g.cn != 3 || g.win_w != W || g.mode != RESIZE_LINEAR) return false;
    const int gpr = W / 4, nh = ctx->split_helpers;
    int       nph = 0, nwc = 0;
    for (int p = 32; p >= 1; p--) {
        const int w = (p * gpr + 63) / 64;
        if (w + nh <= 16) {
            nph = p, nwc = w;
            break;
        }
    }
    if (nph == 0) return false;
    const int rpl = std::max(1, std::min(ctx->split_rpl, kSplitTRMax / nph));
    const int tr  = nph * rpl;
    long      by  = 0;
    for (const J_& g : geo) by = std::max(by, stage_bytes_for(3, stage_rows_for(g, tr), stage_cols(g)));
    by             = (by + 1023) / 1024 * 1024;
    const int lds  = split_lds_layout(W, (int)by).total;
    const int occ  = ctx->split_occ == 2 && !P.tail && lds <= kMaxLds / 2 ? 2 : 1; // (the TAIL form spills at 64 VGPRs)
    if (lds > kMaxLds) return false;
    P.tr          = tr;
    P.stage_bytes = (int)by;
    P.max_win_w   = W;
    P.threads     = (nwc + nh) * 64;
    P.lds         = occ == 2 ? lds : std::max(lds, kMaxLds / 2 + 1024);
    sa.nwc = nwc, sa.nph = nph, sa.rpl = rpl, sa.win_w = W, sa.occ = occ;
    return true;
}

// Direct call (the common case: C2, C5's image, every record transformed straight from its source in
// one launch group): one launch and nothing else on the stream.  The host checks the records, sizes
// the launch from their geometry and writes each record's AugJob (plan_direct) into the slot's
// pinned table; the tile kernel reads the jobs from there itself (an LDS-DMA of one job per tile,
// a tile ahead, over PCIe) -- no planner or upload launch ahead of it.  Returns false (nothing done)
// when some record needs the multi-pass planner: rotation, resize_short, contrast's two passes,
// 2x-area + photometric, the mask gather pass, or records of several launch groups.
template <typename Phase>
bool run_direct(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
                const aeon_aug_params* params, const aeon_out_desc& od, void* out_dev, hipStream_t stream,
                bool is_mask, Phase&& phase)
{
    const OutView        ov = out_view(od);
    const aeon_out_desc& o  = ov.ko; // what the kernels write
    std::vector<JobGeom>& geo = ctx->geoms;
    geo.resize(n);
    std::vector<AugJob>& jobs = ctx->direct_jobs; // each record planned once, copied into the slot below
    if (jobs.size() < (size_t)n) jobs.resize(n);
    int  key = -1, max_h = 0;
    bool vec_ok = !o.fixed_aspect_ratio;
    const OutGeom og = out_geom(o);
    for (int i = 0; i < n; i++) {
        const aeon_img_desc&   d = descs[i];
        const aeon_aug_params& p = params[i];
        if (d.elem_bytes != 0 && d.elem_bytes != 1) return false;
        if (is_mask && d.channels == 1 && o.channels == 1 && p.angle == 0) return false; // mask gather pass
        if (p.angle != 0 || (!is_mask && (p.resize_short_size > 0 || expands(p)))) return false;
        if (!is_mask && p.interp > AEON_INTERP_NEAREST) return false; // CUBIC / AREA / LANCZOS4 (plan_image)
        validate_record(d, p, o, is_mask);
        AugJob& J = jobs[i];
        plan_direct(d, (uint64_t)src_base, p, og, (uint64_t)out_dev + (uint64_t)i * o.item_stride, is_mask, J);
        const int photo = J.photo, mode = J.mode; // (plan_direct: the cv::resize dispatch, photometric flags)
        if ((photo & PHOTO_CONTRAST) || (photo && mode == RESIZE_AREA2X)) return false;
        const bool tail = mode == RESIZE_LINEAR && J.xv < p.out_w * d.channels;
        const int  k    = mode * 4 + (tail ? 2 : 0) + (photo ? 1 : 0);
        if (key < 0) key = k;
        else if (k != key) return false;
        if ((((uint64_t)out_dev + (uint64_t)i * o.item_stride) & 15) != 0 || (p.out_w & 3) != 0) vec_ok = false;
        JobGeom& g = geo[i];
        g.mode = mode, g.cn = d.channels, g.crop_w = p.crop_w, g.crop_h = p.crop_h;
        g.win_w = g.dst_w = p.out_w, g.win_h = g.dst_h = p.out_h, g.photo = photo, g.stats_slot = -1;
        g.scale_x = J.scale_x, g.scale_y = J.scale_y;
        max_h     = std::max(max_h, p.out_h);
    }
    LaunchPlan P;
    P.rm     = key >> 2;
    P.tail   = (key & 2) != 0;
    P.photo  = (key & 1) != 0;
    P.vec_ok = vec_ok;
    P.rtab   = P.photo && o.dtype == AEON_DTYPE_F32;
    // non-photometric INTER_LINEAR into float32 CHW planes, one window width: augment_split (staging on
    // helper waves, split_kernels.hip); else augment_tiles' shape
    SplitArgs  sa{};
    const bool split = ctx->split && !P.photo && P.rm == RESIZE_LINEAR && o.dtype == AEON_DTYPE_F32 && o.channel_major &&
                       vec_ok && !ov.u8_map && !o.fixed_aspect_ratio && plan_split(ctx, geo, P, sa);
    if (!split) P.shape(geo);
    P.max_tiles = (max_h + P.tr - 1) / P.tr;
    // every tile reads its job over PCIe: past ~512 KB of such reads per launch the multi-pass path's
    // device table wins (C5's image launch, 4,096 tiles of 256 B: 98 vs 90 us of kernels per step;
    // C2, 1,792 tiles: direct 3 us faster; a job table the kernel imports itself -- one PCIe read per
    // job into device memory, flags, tiles fetching through L2 -- measured no faster, profiles/r03)
    // (C5's image launch with 128-B hot-half fetches, 512 KB: 112.5 vs 95.5 us per step)
    if ((size_t)P.max_tiles * n * sizeof(AugJob) > kDirectFetchMax) return false;
    phase(2);
    int         slot;
    Slot&       s     = take_slot(ctx, stream, slot);
    phase(3);
    const float* d_lut = resident_lut(ctx, od, ov.u8_map);
    ensure_ring(ctx, (size_t)n * sizeof(AugJob), 16, 32);
    // without photometric stages the tiles read only each job's hot half: the table holds just those
    // (half the bytes the host writes and publishes)
    const size_t stride = P.photo ? sizeof(AugJob) : (size_t)kJobHotBytes;
    const size_t tbytes = (size_t)n * stride;
    // the jobs go straight into the slot's HBM table when it has one (no pinned copy first), else
    // into the pinned slot the tiles read over PCIe
    const bool vram = ctx->vram_jobs && tbytes > 0 && tbytes <= kVramTableMax && tbytes <= s.vram_cap;
    uint8_t*   dstt = vram ? s.vram : s.host;
    // largest crop first: the first round's workgroups take the first jobs' tiles and the dynamic tail
    // hands out the rest in table order, so the cheapest tiles come last and the launch's tail is
    // theirs (each job carries its own source and output: the order changes nothing else)
    // (a counting sort into 32 area classes: two passes, ~1 us for 256 records, where a comparison sort
    // cost the host several)
    std::vector<int>& order = ctx->direct_order;
    order.resize(n);
    {
        int64_t amax = 1;
        for (int i = 0; i < n; i++) amax = std::max(amax, (int64_t)geo[i].crop_w * geo[i].crop_h);
        int  cnt[33] = {0};
        auto cls     = [&](int i) { return 31 - (int)((int64_t)geo[i].crop_w * geo[i].crop_h * 31 / amax); };
        for (int i = 0; i < n; i++) cnt[cls(i) + 1]++;
        for (int c = 0; c < 32; c++) cnt[c + 1] += cnt[c];
        for (int i = 0; i < n; i++) order[cnt[cls(i)]++] = i;
    }
    for (int i = 0; i < n; i++) {
        AugJob& J = jobs[order[i]];
        J.tiles   = (J.win_h + P.tr - 1) / P.tr;
        std::memcpy(dstt + i * stride, &J, stride);
    }
    phase(4);
    const bool timed = ctx->timing && (ctx->timing_calls++ % ctx->timing_every) == ctx->timing_every - 1;
    if (o.fixed_aspect_ratio) // std::fill_n of each item's canvas, its whole byte size (etl_image.cpp:263)
        HIP_OK(hipMemset2DAsync(out_dev, o.item_stride, 0,
                                (size_t)o.canvas_w * o.canvas_h * o.channels * out_elem_bytes(od.dtype), n, stream));
    const uint8_t* vt = vram ? publish_written(s, tbytes) : nullptr;
    phase(5);
    LaunchArgs     a  = launch_args(ctx, s, vt ? vt : s.host_dev, P, n, o, d_lut, 1, ov.u8_map);
    a.job_stride      = (int)stride;
    a.jobs_host       = 1; // (read-through loads: pinned host memory, or the uncached HBM copy)
    // (the algorithmic bytes only for a timed launch: a pass over the records the call does not need)
    const double lbytes = timed ? launch_bytes(geo, KM_FINAL, out_elem_bytes(o.dtype)) : 0;
    if (split) {
        KernelTimer t{};
        if (timed) t = take_timer(ctx, KM_FINAL, lbytes);
        const int grid = std::min(a.total_tiles, sa.occ * ctx->n_cu); // sa.occ workgroups per CU (the LDS request holds it)
        HIP_OK(launch_split(P.tail, sa.occ, a, sa, grid, stream, timed ? t.start : nullptr, timed ? t.stop : nullptr));
        if (timed) ctx->timers.push_back(t);
    } else {
        timed_launch(ctx, KM_FINAL, P, a, stream, lbytes, timed);
    }
    phase(6);
    release_slot(ctx, slot, stream);
    phase(7);
    return true;
}

// Contrast records in ONE launch (record_kernels.hip): every record 3-channel, INTER_LINEAR with no
// OpenCV scalar-tail columns, no rotation / resize_short / expand, one output size that the lanes'
// registers hold (win_w <= 256, a multiple of 4; win_h <= 224), float32 CHW out; some record with
// contrast (else the single-pass direct call is the better one).  The post-hue record stays on chip:
// no u8 intermediate written and read back, no contrast_reduce launch.  Returns false (nothing done)
// for any other call.  AEON_HIP_RECORDS=0 sends such calls through the two-launch path.
template <typename Phase>
bool run_records(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
                 const aeon_aug_params* params, const aeon_out_desc& od, void* out_dev, hipStream_t stream,
                 bool is_mask, Phase&& phase)
{
    if (is_mask || n <= 0 || !ctx->records) return false;
    const OutView        ov = out_view(od);
    const aeon_out_desc& o  = ov.ko;
    if (o.dtype != AEON_DTYPE_F32 || !o.channel_major || o.fixed_aspect_ratio || o.channels != 3) return false;
    if ((((uint64_t)out_dev) & 15) != 0 || (o.item_stride & 15) != 0) return false;
    const int W = params[0].out_w, H = params[0].out_h;
    int       nph = rec_phases(W, H);
    if (ctx->rec_phases > 0 && W / 4 * ctx->rec_phases <= 1024 && (H + ctx->rec_phases - 1) / ctx->rec_phases <= kRecRows)
        nph = ctx->rec_phases; // (development: AEON_HIP_REC_PHASES)
    if (W <= 0 || (W & 3) != 0 || W > 4 * 256 || H <= 0 || nph <= 0) return false;
    if (simd_boundary(W * 3) < W * 3) return false; // OpenCV's scalar row tail
    bool      contrast = false;
    long      stage    = 0;
    JobGeom   g{};
    for (int i = 0; i < n; i++) {
        const aeon_img_desc&   d = descs[i];
        const aeon_aug_params& p = params[i];
        if (d.channels != 3 || (d.elem_bytes != 0 && d.elem_bytes != 1)) return false;
        if (p.angle != 0 || p.resize_short_size > 0 || expands(p) || p.interp != AEON_INTERP_LINEAR) return false;
        if (p.out_w != W || p.out_h != H || p.crop_w <= 0 || p.crop_h <= 0) return false;
        if (choose_mode(p.crop_w, p.crop_h, W, H, AEON_INTERP_LINEAR, 3) != RESIZE_LINEAR) return false;
        contrast |= (photo_flags(p) & PHOTO_CONTRAST) != 0;
        g.mode = RESIZE_LINEAR, g.cn = 3, g.crop_w = p.crop_w, g.crop_h = p.crop_h, g.win_w = W, g.win_h = H;
        g.scale_x = 1. / ((double)W / p.crop_w);
        g.scale_y = 1. / ((double)H / p.crop_h);
        stage     = std::max(stage, stage_bytes_for(3, stage_rows_for(g, nph * kRecTileRows), stage_cols(g)));
    }
    if (!contrast) return false;
    stage         = (stage + 1023) / 1024 * 1024;
    const int lds = rec_lds_layout(W, (int)stage).total;
    if (lds > kMaxLds) return false;
    for (int i = 0; i < n; i++) validate_record(descs[i], params[i], o, false);
    phase(2);
    int   slot;
    Slot& s = take_slot(ctx, stream, slot);
    phase(3);
    const float* d_lut = resident_lut(ctx, od, false);
    ensure_ring(ctx, (size_t)n * sizeof(AugJob), 16, 32);
    AugJob*       jt   = (AugJob*)s.host;
    const OutGeom og   = out_geom(o);
    bool          fast = true;
    double        bytes = 0;
    for (int i = 0; i < n; i++) {
        plan_direct(descs[i], (uint64_t)src_base, params[i], og, (uint64_t)out_dev + (uint64_t)i * o.item_stride, false,
                    jt[i]);
        if ((jt[i].photo & PHOTO_BS) && jt[i].bs_kind != BS_FIXPT) fast = false;
        // algorithmic bytes: the crop read once + the float32 output written once
        bytes += (double)params[i].crop_w * params[i].crop_h * 3 + (double)W * H * 3 * 4;
    }
    phase(4);
    const uint8_t* vt = publish_table(ctx, s, (size_t)n * sizeof(AugJob));
    phase(5);
    LaunchArgs a{};
    a.jobs        = (const AugJob*)(vt ? vt : s.host_dev);
    a.jobs_host   = 1; // (read-through loads: pinned host memory, or the uncached HBM copy)
    a.job_bytes   = (int)sizeof(AugJob);
    a.lut         = d_lut;
    a.hsv_tables  = ctx->d_hsv;
    a.error       = ctx->call_error;
    a.stage_bytes = (int)stage;
    a.max_win_w   = W;
    a.out_dtype   = AEON_DTYPE_F32;
    a.channel_major = 1;
    a.bgr_to_rgb  = o.bgr_to_rgb && o.channels == 3;
    a.threads     = (nph * (W / 4) + 63) / 64 * 64;
    // helper waves (record_kernels.hip: staging only) when the workgroup has room for them
    const bool split = ctx->rec_helpers > 0 && a.threads + 64 * ctx->rec_helpers <= 1024;
    if (split) a.threads += 64 * ctx->rec_helpers;
    a.lds_bytes   = lds;
#ifdef AEON_HIP_TRACE
    a.trace = ctx->trace; // development builds only (tools/trace_records.py)
#endif
    const RecArgs r{n, nph, W, H, ((H + nph - 1) / nph + kRecTileRows - 1) / kRecTileRows};
    const int     grid  = std::min(n, ctx->n_cu); // one workgroup per CU (LDS, 14-16 waves at <= 128 VGPRs)
    const bool    timed = ctx->timing && (ctx->timing_calls++ % ctx->timing_every) == ctx->timing_every - 1;
    KernelTimer   t{};
    if (timed) t = take_timer(ctx, KM_FINAL, bytes);
    HIP_OK(launch_contrast_records(fast, split, a, r, grid, stream, timed ? t.start : nullptr, timed ? t.stop : nullptr));
    if (timed) ctx->timers.push_back(t);
    phase(6);
    release_slot(ctx, slot, stream);
    phase(7);
    return true;
}

// The masks of an image + mask call (aeon_hip_augment_pair_batch): 8-bit single-channel records
// without rotation into uint8 items, sharing the images' params.
struct MaskSet {
    const aeon_img_desc* descs;
    const void*          src_base;
    aeon_out_desc        out;
    void*                out_dev;
};

int run_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
              const aeon_aug_params* params, const aeon_out_desc* out, void* out_dev, void* stream_,
              bool is_mask, const MaskSet* ms = nullptr)
{
    if (!ctx || n < 0 || (n > 0 && (!descs || !params || !out || !out_dev || !src_base)))
        fail(AEON_HIP_EINVAL, "null argument");
    if (n == 0) return 0;
    if (n > 65535) fail(AEON_HIP_EINVAL, "at most 65535 records per call");
    const aeon_out_desc& od = *out; // as declared; `o` below is what the kernels write (out_view)
    if (od.dtype < AEON_DTYPE_U8 || od.dtype > AEON_DTYPE_F64) fail(AEON_HIP_EUNSUPPORTED, "unknown output dtype");
    if (od.has_mean && od.dtype != AEON_DTYPE_F32 && od.dtype != AEON_DTYPE_F64)
        fail(AEON_HIP_EINVAL,
             "Standardization (mean, stddev) is supported only for float or double 'output_type'.");
    const OutView        ov = out_view(od);
    const aeon_out_desc& o  = ov.ko;
    if (o.bgr_to_rgb && o.channels != 3)
        fail(AEON_HIP_EINVAL, "invalid config: bgr_to_rgb can be 'true' only for channels set to '3'");
    // pixel_mask / depthmap loaders never standardize or swap channels (etl_pixel_mask.cpp:94-105,
    // etl_depthmap.cpp:98-134): refuse both, so rotated and unrotated masks agree
    if (is_mask && (od.has_mean || od.bgr_to_rgb))
        fail(AEON_HIP_EINVAL, "pixel masks / depth maps take no mean/stddev and no bgr_to_rgb");
    if (od.fixed_aspect_ratio) {
        // aeon's fixed-aspect loader zeroes the item's whole byte size and views the canvas as
        // CV_8U planes whatever the output type (etl_image.cpp:263-305): out_view
        if (od.canvas_w <= 0 || od.canvas_h <= 0 ||
            (size_t)od.canvas_w * od.canvas_h * od.channels * out_elem_bytes(od.dtype) > od.item_stride)
            fail(AEON_HIP_EINVAL, "fixed_aspect_ratio: canvas does not fit item_stride");
    }
    hipStream_t stream = (hipStream_t)stream_;

    std::lock_guard<std::mutex> lock(ctx->mu);
    ctx->call_error = stream_error(ctx, stream);
    using clk = std::chrono::steady_clock;
    auto t_prev = clk::now();
    auto phase  = [&](int k) {
        if (!ctx->host_profile) return;
        auto t = clk::now();
        ctx->host_ns[k].push_back(std::chrono::duration<double, std::nano>(t - t_prev).count());
        t_prev = t;
    };
    HIP_OK(hipSetDevice(ctx->device));
    phase(0);
    // (a pair call goes through the planner: its masks join the images' launch)
    if (!ms && ctx->direct && run_direct(ctx, n, descs, src_base, params, od, out_dev, stream, is_mask, phase))
        return 0;
    if (!ms && run_records(ctx, n, descs, src_base, params, od, out_dev, stream, is_mask, phase)) return 0;

    LaunchPlan             pre_all, pre2_all, pass1_all, main_all;
    GrPlan                 gr_short, gr_main;
    std::vector<RotJob>    rot;
    std::vector<ExpandJob> exp;
    std::vector<Mask16Job> m16;
    size_t     scratch_bytes = 0;
    for (int i = 0; i < n; i++) {
        uint8_t* item = (uint8_t*)out_dev + (size_t)i * o.item_stride;
        // pixel masks without rotation (and every 16-bit record): the NEAREST gather pass
        const bool gather = descs[i].elem_bytes == 2 ||
                            (is_mask && descs[i].channels == 1 && o.channels == 1 && params[i].angle == 0 &&
                             (descs[i].elem_bytes == 0 || descs[i].elem_bytes == 1));
        if (gather) plan_mask16(descs[i], src_base, params[i], o, item, is_mask, m16, rot, scratch_bytes);
        else if (descs[i].elem_bytes == 0 || descs[i].elem_bytes == 1)
            plan_image(descs[i], src_base, params[i], o, item, is_mask, rot, exp, gr_short, pre_all, gr_main, pre2_all,
                       pass1_all, main_all, scratch_bytes);
        else fail(AEON_HIP_EINVAL, "elem_bytes must be 1 (CV_8U) or 2 (CV_16U)");
    }
    for (int i = 0; ms && i < n; i++) // the pair call's masks: the gather pass's jobs
        plan_mask16(ms->descs[i], ms->src_base, params[i], ms->out, (uint8_t*)ms->out_dev + (size_t)i * ms->out.item_stride,
                    true, m16, rot, scratch_bytes);

    phase(1);
    // one launch per (resize mode, photometric) group: the kernels are specialised on both
    // one launch per (resize mode, scalar tail, photometric) group: the kernels are specialised
    // on all three
    auto has_tail = [](const AugJob& J) { return J.mode == RESIZE_LINEAR && J.xv < J.dst_w * J.cn; };
    std::vector<LaunchPlan> pre(8), pre2(8), pass1(8), main(16);
    for (int g = 0; g < 8; g++) {
        pre[g].rm = pre2[g].rm = pass1[g].rm = g >> 1;
        pre[g].tail = pre2[g].tail = pass1[g].tail = (g & 1) != 0;
        pass1[g].photo = true;
    }
    for (int g = 0; g < 16; g++) main[g].rm = g >> 2, main[g].tail = (g & 2) != 0, main[g].photo = (g & 1) != 0;
    for (const AugJob& J : pre_all.jobs) pre[J.mode * 2 + has_tail(J)].jobs.push_back(J);
    for (const AugJob& J : pre2_all.jobs) pre2[J.mode * 2 + has_tail(J)].jobs.push_back(J);
    for (const AugJob& J : pass1_all.jobs) pass1[J.mode * 2 + has_tail(J)].jobs.push_back(J);
    for (const AugJob& J : main_all.jobs) main[J.mode * 4 + has_tail(J) * 2 + (J.photo ? 1 : 0)].jobs.push_back(J);
    const size_t     rot_off   = 0;
    const size_t     m16_off   = rot_off + rot.size() * sizeof(RotJob);
    const size_t     exp_off   = m16_off + m16.size() * sizeof(Mask16Job);
    size_t           blob      = exp_off + exp.size() * sizeof(ExpandJob);
    for (GrPlan* g : {&gr_short, &gr_main}) { // jobs, then their Lanczos taps (offsets made absolute)
        if (g->jobs.empty()) continue;
        if (g->n_taps > 4096 && !ctx->plan_pool) ctx->plan_pool.reset(new thread_pool(thread_affinity_map("")));
        g->finalize();
        blob        = (blob + 15) & ~(size_t)15;
        g->off      = blob;
        blob += g->jobs.size() * sizeof(ResizeJob);
        g->lz_off = blob;
        blob += g->n_taps * sizeof(LzIn);
    }
    blob = (blob + 15) & ~(size_t)15;
    int              exp_max_px = 0;
    for (const ExpandJob& E : exp) exp_max_px = std::max(exp_max_px, E.ew * E.eh);
    int              m16_max_h = 0, m16_max_w = 0, m16_max_seg = 0;
    double           m16_bytes = 0; // algorithmic: crop read once + output written once
    for (const Mask16Job& M : m16) {
        m16_max_h = std::max(m16_max_h, M.out_h), m16_max_w = std::max(m16_max_w, M.out_w);
        m16_max_seg = std::max(m16_max_seg, M.crop_w * M.src_elem);
        m16_bytes += (double)M.crop_w * M.crop_h * M.src_elem + (double)M.out_w * M.out_h * out_elem_bytes(M.dtype);
    }
    // distinct source rows of any block of the gather pass: the kernel's own row map
    // (sy = min(floor(y * ify), crop_h - 1), monotonic in y), evaluated at each block's ends
    int m16_max_slots = 1;
    if (!m16.empty()) {
        const int srows = mask16_rows(m16_max_w, m16_max_seg);
        for (const Mask16Job& M : m16)
            for (int y0 = 0; y0 < M.out_h; y0 += srows) {
                const auto sy = [&](int y) { return std::min((int)std::floor(y * M.scale_y), M.crop_h - 1); };
                const int  y1 = std::min(y0 + srows, M.out_h) - 1;
                m16_max_slots = std::max(m16_max_slots, std::min(y1 - y0 + 1, sy(y1) - sy(y0) + 1));
            }
    }
    int              rot_max_tiles = 0, rot_words = 0, rot_cn = rot.empty() ? 0 : rot[0].cn; // (rotate_tiles)
    for (size_t r = 0; r < rot.size(); r++) {
        const RotJob& R = rot[r];
        if (R.cn != rot_cn) rot_cn = 0;
        rot_max_tiles   = std::max(rot_max_tiles, ((R.ow + 63) / 64) * ((R.oh + 31) / 32));
        rot_words       = std::max(rot_words, rot_box_words(R.angle));
    }
    std::vector<int> slot_tiles(pass1_all.jobs.size(), 0);
    int              partial_stride = 1;
    for (auto* v : {&pre, &pre2, &pass1, &main})
        for (LaunchPlan& P : *v) {
            if (P.jobs.empty()) continue;
            P.vec_ok = main_all.vec_ok;
            P.rtab   = v == &main && P.photo && o.dtype == AEON_DTYPE_F32;
            // final non-photometric INTER_LINEAR float32 CHW launches (C5's images): augment_split
            P.split = v == &main && ctx->split && !P.photo && P.rm == RESIZE_LINEAR && o.dtype == AEON_DTYPE_F32 &&
                      o.channel_major && P.vec_ok && !ov.u8_map && !o.fixed_aspect_ratio && !(ms && ctx->fuse_masks) &&
                      plan_split(ctx, P.jobs, P, P.sa);
            P.finalize();
            P.blob_off = blob;
            blob += P.jobs.size() * sizeof(AugJob);
            if (v == &pass1)
                for (const AugJob& J : P.jobs) {
                    slot_tiles[J.stats_slot] = J.tiles;
                    partial_stride           = std::max(partial_stride, J.tiles * 8); // (tile, wave) sums
                }
            if (v == &main)
                for (AugJob& J : P.jobs)
                    if (J.stats_slot >= 0) J.stats_tiles = slot_tiles[J.stats_slot];
        }
    const size_t partial_words = std::max<size_t>(4, pass1_all.jobs.size() * partial_stride * 4);
    // the Lanczos4 taps the device builds: after everything the host writes (not uploaded)
    size_t table_cap = (blob + 15) & ~(size_t)15;
    for (GrPlan* g : {&gr_short, &gr_main}) {
        if (g->n_taps == 0) continue;
        g->taps_off = table_cap;
        table_cap += ((g->n_taps * sizeof(GrTap)) + 15) & ~(size_t)15;
        for (ResizeJob& R : g->jobs)
            if (R.method == GR_LANCZOS4) R.coef_x += (int32_t)g->taps_off, R.coef_y += (int32_t)g->taps_off;
    }

    phase(2);
    int   slot;
    Slot& s = take_slot(ctx, stream, slot);
    phase(3);
    const float* d_lut = resident_lut(ctx, od, ov.u8_map);
    // job tables, contrast sums and shifts: one capacity for every slot of the ring (a call never
    // allocates unless it needs more than any call before it); scratch per slot, on demand
    // (sized for the Lanczos4 taps with no axis shared: the shared count varies from call to call, and a
    // ring growth inside a loader's steady state costs ~10-20 ms of allocations)
    size_t ring_need = table_cap;
    for (GrPlan* g : {&gr_short, &gr_main})
        ring_need += (g->n_taps_max - g->n_taps) * (sizeof(LzIn) + sizeof(GrTap)) + 32;
    ensure_ring(ctx, ring_need, partial_words * 4, std::max<size_t>(1, pass1_all.jobs.size()) * 4 * sizeof(double));
    if (scratch_bytes > s.scratch_cap) grow(s.scratch, s.scratch_cap, scratch_bytes + scratch_bytes / 4, false); // (slack as ensure_ring)
    for (RotJob& R : rot) R.out_ptr += (uint64_t)s.scratch;
    for (Mask16Job& M : m16)
        if (M.src_scratch) M.src_ptr += (uint64_t)s.scratch;
    for (ExpandJob& E : exp) {
        E.out_ptr += (uint64_t)s.scratch;
        if (E.src_scratch) E.src_ptr += (uint64_t)s.scratch;
    }
    if (!exp.empty()) std::memcpy(s.host + exp_off, exp.data(), exp.size() * sizeof(ExpandJob));
    for (GrPlan* g : {&gr_short, &gr_main}) {
        if (g->jobs.empty()) continue;
        for (ResizeJob& R : g->jobs) {
            if (R.src_scratch) R.src_ptr += (uint64_t)s.scratch;
            if (R.out_scratch) R.out_ptr += (uint64_t)s.scratch;
        }
        std::memcpy(s.host + g->off, g->jobs.data(), g->jobs.size() * sizeof(ResizeJob));
        if (g->n_taps) g->fill_taps(ctx->plan_pool.get(), (LzIn*)(s.host + g->lz_off));
    }
    if (!rot.empty()) std::memcpy(s.host + rot_off, rot.data(), rot.size() * sizeof(RotJob));
    if (!m16.empty()) std::memcpy(s.host + m16_off, m16.data(), m16.size() * sizeof(Mask16Job));
    for (auto* v : {&pre, &pre2, &pass1, &main})
        for (LaunchPlan& P : *v) {
            for (AugJob& J : P.jobs) { // relocate scratch references
                if (v != &main) J.out_ptr += (uint64_t)s.scratch;
                if (J.src_scratch) J.src_ptr += (uint64_t)s.scratch;
            }
            if (!P.jobs.empty()) std::memcpy(s.host + P.blob_off, P.jobs.data(), P.jobs.size() * sizeof(AugJob));
        }
    phase(4);
    // Job-table transport: tables up to kUploadKernelMax go up by a small kernel on the launch
    // stream that reads the pinned slot over PCIe (kernel-to-kernel order, no cross-queue wait:
    // 43.5 vs 44.2 us per C2 step against an SDMA copy + event, which costs a ~6.6 us dispatch gap);
    // larger ones by SDMA on copy_stream, which overlaps the previous call's kernels while the
    // upload kernel would read PCIe at ~34 GB/s (C3, 512 KB: 347 vs 357 us per step).
    // A call of pixel-mask gather jobs only (C5's masks): the gather reads its few jobs (one per
    // workgroup) from the pinned slot itself, no upload launch ahead of it.
    bool mask_only = !m16.empty() && rot.empty() && exp.empty() && gr_short.jobs.empty() && gr_main.jobs.empty();
    for (auto* v : {&pre, &pre2, &pass1, &main})
        for (LaunchPlan& P : *v) mask_only = mask_only && P.jobs.empty();
    // the tables in HBM written by the host (no upload launch) unless a LANCZOS4 tap table is among
    // them (read per output pixel: the cached device copy)
    const bool     vram_ok = gr_short.n_taps == 0 && gr_main.n_taps == 0;
    const uint8_t* vt      = vram_ok ? publish_table(ctx, s, blob) : nullptr;
    const uint8_t* table   = vt ? vt : mask_only ? s.host_dev : s.dev;
    // timing events on one call in timing_every (each event pair costs GPU time between launches)
    const bool timed = ctx->timing && (ctx->timing_calls++ % ctx->timing_every) == ctx->timing_every - 1;
    auto launch_masks = [&](const uint8_t* tbl) { // the gather pass, its jobs at tbl + m16_off
        KernelTimer t{};
        if (timed) t = take_timer(ctx, KM_FINAL, m16_bytes);
        HIP_OK(launch_nearest((const Mask16Job*)(tbl + m16_off), (int)m16.size(), m16_max_h, m16_max_w, m16_max_seg,
                              m16_max_slots, stream, timed ? t.start : nullptr, timed ? t.stop : nullptr));
        if (timed) ctx->timers.push_back(t);
    };
    // (A pair call's tables go up together by the upload kernel, and its gather launch reads the device
    // copy: C5 93-94 us per step against 96-98 for the image and mask calls, whose gather reads the
    // pinned slot -- 4.5 us more kernel time -- and 97-98 for the masks first on the pinned slot while
    // SDMA uploads the images' table; tools/c5_ab.sh)
    if (mask_only || vt) {
    } else if (blob > kUploadKernelMax) {
        HIP_OK(hipMemcpyAsync(s.dev, s.host, blob, hipMemcpyHostToDevice, ctx->copy_stream));
        HIP_OK(hipEventRecord(s.copied, ctx->copy_stream));
        HIP_OK(hipStreamWaitEvent(stream, s.copied, 0));
    } else {
        HIP_OK(launch_upload_table(s.host_dev, s.dev, blob, stream));
    }
    for (GrPlan* g : {&gr_short, &gr_main}) // the Lanczos4 taps from their host-computed inputs
        if (g->n_taps)
            HIP_OK(launch_lanczos4_taps((const LzIn*)(table + g->lz_off), (GrTap*)(table + g->taps_off), (int)g->n_taps,
                                        stream));
    phase(5);

    auto args = [&](const LaunchPlan& L) {
        return launch_args(ctx, s, table, L, (int)L.jobs.size(), o, d_lut, partial_stride, ov.u8_map);
    };
    const size_t oelem = out_elem_bytes(o.dtype);
    if (o.fixed_aspect_ratio) // std::fill_n of each item's canvas, its whole byte size (etl_image.cpp:263)
        HIP_OK(hipMemset2DAsync(out_dev, o.item_stride, 0,
                                (size_t)o.canvas_w * o.canvas_h * o.channels * out_elem_bytes(od.dtype), n, stream));
    if (!rot.empty()) // image::rotate pre-pass first: the gather and tile passes read its output
        HIP_OK(launch_rotate((const RotJob*)(table + rot_off), (int)rot.size(), rot_max_tiles, rot_words, rot_cn, ctx->call_error,
                             stream));
    if (!exp.empty()) // then image::expand (etl_image.cpp:155-159)
        HIP_OK(launch_expand((const ExpandJob*)(table + exp_off), (int)exp.size(), exp_max_px, stream));
    // A pair call whose images are one tile launch: the masks' row blocks go into that launch (its
    // workgroups take them after their tiles, augment_kernels.hip mask_blocks) -- no gather launch.
    LaunchPlan* fused = nullptr;
    LaunchArgs  fused_masks{};
    if (ms && ctx->fuse_masks && !m16.empty() && rot.empty() && exp.empty() && gr_short.jobs.empty() && gr_main.jobs.empty()) {
        int groups = 0;
        for (auto* v : {&pre, &pre2, &pass1, &main})
            for (LaunchPlan& P : *v)
                if (!P.jobs.empty()) groups++, fused = &P;
#ifndef AEON_HIP_FUSED_MASK_ROWS
#define AEON_HIP_FUSED_MASK_ROWS 64
#endif
        const int srows = std::min(mask16_rows(m16_max_w, m16_max_seg), AEON_HIP_FUSED_MASK_ROWS);
        bool in_main = false;
        for (LaunchPlan& P : main) in_main |= fused == &P;
        if (groups == 1 && in_main && srows >= 1 && !fused->has_contrast && !fused->split) {
            const int pitch = mask16_pitch(m16_max_seg);
            const int slots = std::max(1, std::min(m16_max_slots, srows));
            const int base  = lds_layout(fused->max_win_w, fused->tr, fused->stage_bytes, fused->photo && fused->has_hue,
                                         fused->rtab).stage;
            const int need  = base + kMaskBlockHdrBytes + slots * pitch;
            fused_masks.mjobs    = (const Mask16Job*)(table + m16_off);
            fused_masks.m_ctr    = ctx->d_tail + aeon_hip_ctx::kSlots + slot;
            fused_masks.m_bpj    = (m16_max_h + srows - 1) / srows;
            fused_masks.m_blocks = (int)m16.size() * fused_masks.m_bpj;
            fused_masks.m_rows = srows, fused_masks.m_pitch = pitch, fused_masks.m_perm = 1, fused_masks.m_slots = slots;
            fused_masks.m_lds    = base;
            fused_masks.lds_bytes = std::max(fused->lds, need);
            if (fused_masks.lds_bytes > kMaxLds) fused = nullptr;
        } else {
            fused = nullptr;
        }
    }
    if (!m16.empty() && !fused) launch_masks(table);
    auto generic = [&](const GrPlan& g) {
        if (g.jobs.empty()) return;
        KernelTimer t{};
        if (timed) t = take_timer(ctx, KM_RAW, g.bytes);
        if (timed) HIP_OK(hipEventRecord(t.start, stream));
        const int gbgr = o.bgr_to_rgb && o.channels == 3, gchm = o.channel_major;
        for (const GrPlan::Sub& u : g.subs) {
            const ResizeJob* gj   = (const ResizeJob*)(table + g.off) + u.first;
            const float*     glut = u.any_final ? d_lut : nullptr;
            if (u.sep)
                HIP_OK(launch_resize_sep(u.sep, u.area, gj, table, u.count, u.max_tiles, u.TR, u.CW, u.NR, u.SW, u.cn_max, glut, gbgr,
                                         gchm, ctx->call_error, stream));
            else
                HIP_OK(launch_resize_generic(gj, table, u.count, u.max_tiles, u.TR, u.CW, u.NR, u.xs, u.amax, u.cn_max, u.SW,
                                             glut, gbgr, gchm, ctx->call_error, stream));
        }
        if (timed) {
            HIP_OK(hipEventRecord(t.stop, stream));
            ctx->timers.push_back(t);
        }
    };
    generic(gr_short);
    for (LaunchPlan& P : pre)
        if (!P.jobs.empty()) timed_launch(ctx, KM_RAW, P, args(P), stream, launch_bytes(P.jobs, KM_RAW, 1), timed);
    generic(gr_main);
    for (LaunchPlan& P : pre2)
        if (!P.jobs.empty()) timed_launch(ctx, KM_RAW, P, args(P), stream, launch_bytes(P.jobs, KM_RAW, 1), timed);
    for (LaunchPlan& P : pass1)
        if (!P.jobs.empty())
            timed_launch(ctx, KM_STATS, P, args(P), stream, launch_bytes(P.jobs, KM_STATS, oelem), timed);
    for (LaunchPlan& P : main) {
        if (P.jobs.empty()) continue;
        if (P.has_contrast) HIP_OK(launch_contrast_reduce(args(P), (int)P.jobs.size(), stream));
        LaunchArgs a     = args(P);
        double     bytes = launch_bytes(P.jobs, KM_FINAL, oelem);
        if (&P == fused) {
            a.mjobs = fused_masks.mjobs, a.m_ctr = fused_masks.m_ctr, a.m_blocks = fused_masks.m_blocks;
            a.m_bpj = fused_masks.m_bpj, a.m_rows = fused_masks.m_rows, a.m_pitch = fused_masks.m_pitch;
            a.m_perm = fused_masks.m_perm, a.m_slots = fused_masks.m_slots, a.m_lds = fused_masks.m_lds;
            a.lds_bytes = fused_masks.lds_bytes;
            bytes += m16_bytes;
        }
        if (P.split) {
            KernelTimer t{};
            if (timed) t = take_timer(ctx, KM_FINAL, bytes);
            HIP_OK(launch_split(P.tail, P.sa.occ, a, P.sa, std::min(a.total_tiles, P.sa.occ * ctx->n_cu), stream,
                                timed ? t.start : nullptr, timed ? t.stop : nullptr));
            if (timed) ctx->timers.push_back(t);
        } else {
            timed_launch(ctx, KM_FINAL, P, a, stream, bytes, timed);
        }
    }
    phase(6);
    release_slot(ctx, slot, stream);
    phase(7);
    return 0;
}

// std::minstd_rand0 whose state word can be read back (an LCG's state is its last output).
struct TrackedEngine {
    using result_type = std::minstd_rand0::result_type;
    std::minstd_rand0 e;
    result_type       last;
    static constexpr result_type min() { return std::minstd_rand0::min(); }
    static constexpr result_type max() { return std::minstd_rand0::max(); }
    explicit TrackedEngine(uint32_t s) : e(s), last(s % 2147483647u == 0 ? 1 : s % 2147483647u) {}
    result_type operator()() { return last = e(); }
};

template <typename F>
int guarded(F&& f)
{
    try {
        return f();
    } catch (const aeon_error& e) {
        g_err = e.what();
        return e.code;
    } catch (const jpeg_error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::invalid_argument& e) {
        g_err = e.what();
        return AEON_HIP_EINVAL;
    } catch (const std::exception& e) {
        g_err = e.what();
        return AEON_HIP_ERUNTIME;
    }
}

} // namespace

namespace aeon_hip {
// The owning decoder's pool runs the context's JPEG entropy decoding (set before the first JPEG call).
void ctx_share_pool(aeon_hip_ctx* ctx, thread_pool* pool)
{
    if (ctx && !ctx->jpeg) ctx->host_pool = pool;
}
} // namespace aeon_hip

extern "C" {

int aeon_hip_ctx_create(int device, aeon_hip_ctx** out)
{
    return guarded([&] {
        if (!out) fail(AEON_HIP_EINVAL, "null out");
        auto* c   = new aeon_hip_ctx();
        c->device = device;
        try {
            HIP_OK(hipSetDevice(device));
            HIP_OK(set_kernel_lds_limit(kMaxLds));
            HIP_OK(contrast_records_lds_limit(kMaxLds));
            HIP_OK(split_lds_limit(kMaxLds));
            HIP_OK(hipMalloc((void**)&c->d_error, sizeof(int32_t) * aeon_hip_ctx::kErrWords));
            HIP_OK(hipMemset(c->d_error, 0, sizeof(int32_t) * aeon_hip_ctx::kErrWords));
            // per slot: the dynamic-tail counter, then (kSlots on) the mask-block counter of pair calls
            HIP_OK(hipMalloc((void**)&c->d_tail, 2 * aeon_hip_ctx::kSlots * sizeof(uint32_t)));
            HIP_OK(hipMemset(c->d_tail, 0, 2 * aeon_hip_ctx::kSlots * sizeof(uint32_t)));
            HIP_OK(hipDeviceSynchronize());
            // RGB2HSV_b division tables (hsv_shift = 12), as OpenCV builds them, then per uchar H
            // HSV2RGB_f's sector fraction f (its own float operations) turned into the weight w of
            // each output channel in t = v*(1 - s*w): t0 w=0, t1 w=1, t2 w=f, t3 w=1-f
            int32_t tab[kHsvWords];
            tab[0] = tab[256] = 0;
            for (int i = 1; i < 256; i++) {
                tab[i]       = cv_round((255 << 12) / (1. * i));
                tab[256 + i] = cv_round((180 << 12) / (6. * i));
            }
            static const int sector_data[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
            for (int H = 0; H < 256; H++) {
                volatile float hf = (float)H;
                hf = hf * (6.f / 180.f);
                while (hf >= 6.f) hf = hf - 6.f;
                int sector = (int)std::floor((float)hf);
                hf         = hf - (float)sector;
                if ((unsigned)sector >= 6u) sector = 0, hf = 0.f;
                const float f      = hf;
                const float wt[4]  = {0.f, 1.f, f, 1.f - f};
                const float w[4]   = {wt[sector_data[sector][0]], wt[sector_data[sector][1]], wt[sector_data[sector][2]], 0.f};
                std::memcpy(&tab[512 + 4 * H], w, sizeof(w));
            }
            HIP_OK(hipMalloc((void**)&c->d_hsv, sizeof(tab)));
            HIP_OK(hipMemcpy(c->d_hsv, tab, sizeof(tab), hipMemcpyHostToDevice));
            for (Slot& s : c->slots) {
                // the ring's completion events only tell the host that the GPU is done reading a
                // slot: no system-scope fence needed (each one idled the GPU ~6 us between launches)
#ifndef AEON_HIP_DONE_FENCE
#define AEON_HIP_DONE_FENCE 0
#endif
                HIP_OK(hipEventCreateWithFlags(&s.done, hipEventDisableTiming |
                                                            (AEON_HIP_DONE_FENCE ? 0 : hipEventDisableSystemFence)));
                // s.copied orders the SDMA job-table upload (copy_stream) before the kernels that read
                // it on the launch stream: it keeps the system-scope release
                HIP_OK(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
            }
            HIP_OK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
            // job tables in HBM written by the host when the GPU exposes all of its memory through
            // the PCIe BAR (else pinned host tables, read over PCIe)
            int large_bar = 0;
            if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) != hipSuccess) large_bar = 0;
            c->vram_jobs = large_bar != 0;
            if (const char* e = std::getenv("AEON_HIP_VRAM_JOBS")) c->vram_jobs = c->vram_jobs && std::atoi(e) != 0;
            // the ring at the size a 512-record call needs (job tables of 128 KB), so steady-state
            // calls of that size never allocate
            ensure_ring(c, 128 * 1024, 64 * 1024, 8 * 1024);
            // diagnostics: host time per phase (printed at destroy); the multi-pass path for every call
            if (const char* e = std::getenv("AEON_HIP_HOST_PROFILE")) c->host_profile = std::atoi(e) != 0;
            if (c->host_profile) std::fprintf(stderr, "[aeon_hip] job tables in HBM (BAR writes): %d\n", (int)c->vram_jobs);
            if (const char* e = std::getenv("AEON_HIP_DIRECT")) c->direct = std::atoi(e) != 0;
            if (const char* e = std::getenv("AEON_HIP_RECORDS")) c->records = std::atoi(e) != 0;
            if (const char* e = std::getenv("AEON_HIP_REC_HELPERS")) c->rec_helpers = std::max(0, std::min(4, std::atoi(e)));
            if (const char* e = std::getenv("AEON_HIP_REC_PHASES")) c->rec_phases = std::atoi(e);
            if (const char* e = std::getenv("AEON_HIP_SPLIT")) c->split = std::atoi(e) != 0;
            if (const char* e = std::getenv("AEON_HIP_SPLIT_HELPERS")) c->split_helpers = std::max(1, std::min(4, std::atoi(e)));
            if (const char* e = std::getenv("AEON_HIP_SPLIT_RPL")) c->split_rpl = std::max(1, std::min(4, std::atoi(e)));
            if (const char* e = std::getenv("AEON_HIP_SPLIT_OCC")) c->split_occ = std::max(1, std::min(2, std::atoi(e)));
            if (const char* e = std::getenv("AEON_HIP_JPEG_HUFF")) c->jpeg_gpu_huff = std::strcmp(e, "host") != 0;
            if (const char* e = std::getenv("AEON_HIP_FUSE_MASKS")) c->fuse_masks = std::atoi(e) != 0;
#ifdef AEON_HIP_TRACE
            // development builds only: s_memtime phase stamps of the tile kernel into this device buffer
            if (const char* e = std::getenv("AEON_HIP_TRACE_PTR")) c->trace = (uint32_t*)std::strtoull(e, nullptr, 0);
#endif
            HIP_OK(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
        return 0;
    });
}

int aeon_hip_ctx_destroy(aeon_hip_ctx* c)
{
    return guarded([&] {
        if (!c) return 0;
        if (c->host_profile && c->host_calls) {
            static const char* names[8] = {"set_device", "plan", "group+finalize", "slot_wait",
                                           "blob_fill", "h2d+wait_event (direct: table publish)", "launches",
                                           "done_event"};
            std::fprintf(stderr, "[aeon_hip host profile] %ld calls, us per call (median/mean/p90):", c->host_calls);
            double total = 0;
            for (int k = 0; k < 8; k++) {
                std::vector<double> v = c->host_ns[k];
                if (v.empty()) continue;
                double sum = 0;
                for (double x : v) sum += x;
                total += sum / v.size();
                std::sort(v.begin(), v.end());
                std::fprintf(stderr, " %s=%.1f/%.1f/%.1f", names[k], v[v.size() / 2] / 1e3, sum / v.size() / 1e3,
                             v[v.size() * 9 / 10] / 1e3);
            }
            std::fprintf(stderr, "; mean total %.1f us\n", total / 1e3);
        }
        (void)hipSetDevice(c->device);
        jpeg_state_destroy(c->jpeg);
        if (!c->open_slots.empty()) (void)hipStreamSynchronize(c->open_stream);
        for (Slot& s : c->slots)
            if (s.pending) (void)hipEventSynchronize(c->slots[s.cover].done);
        for (Slot& s : c->slots) {
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.copied) (void)hipEventDestroy(s.copied);
            if (s.host) (void)hipHostFree(s.host);
            if (s.dev) (void)hipFree(s.dev);
            if (s.vram) free_vram(s.vram, s.vram_cap);
            if (s.scratch) (void)hipFree(s.scratch);
            if (s.partials) (void)hipFree(s.partials);
            if (s.shifts) (void)hipFree(s.shifts);
        }
        for (auto* v : {&c->timers, &c->free_timers})
            for (KernelTimer& t : *v) (void)hipEventDestroy(t.start), (void)hipEventDestroy(t.stop);
        if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
        for (auto& L : c->luts) (void)hipFree(L.dev);
        if (c->d_error) (void)hipFree(c->d_error);
        if (c->d_tail) (void)hipFree(c->d_tail);
        if (c->d_hsv) (void)hipFree(c->d_hsv);
        delete c;
        return 0;
    });
}

int aeon_hip_transpose_batch(aeon_hip_ctx* ctx, const void* src_dev, void* dst_dev, int64_t rows, int64_t cols,
                             int element_size, void* stream)
{
    return guarded([&] {
        if (!ctx || !src_dev || !dst_dev) fail(AEON_HIP_EINVAL, "null argument");
        if (rows < 0 || cols < 0) fail(AEON_HIP_EINVAL, "negative matrix size");
        if (element_size != 1 && element_size != 2 && element_size != 4 && element_size != 8)
            fail(AEON_HIP_EINVAL, "unsupported datatype for transpose");
        if (rows / 64 >= 65535) fail(AEON_HIP_EINVAL, "too many rows for one transpose");
        if (rows == 0 || cols == 0) return 0;
        const uint8_t* s = (const uint8_t*)src_dev;
        uint8_t*       d = (uint8_t*)dst_dev;
        const size_t   bytes = (size_t)rows * cols * element_size;
        if (s < d + bytes && d < s + bytes) fail(AEON_HIP_EINVAL, "transpose buffers overlap");
        std::lock_guard<std::mutex> lock(ctx->mu);
        HIP_OK(hipSetDevice(ctx->device));
        HIP_OK(launch_transpose(src_dev, dst_dev, rows, cols, element_size, (hipStream_t)stream));
        return 0;
    });
}

int aeon_hip_augment_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
                           const aeon_aug_params* params, const aeon_out_desc* out, void* out_dev,
                           void* stream)
{
    return guarded([&] { return run_batch(ctx, n, descs, src_base, params, out, out_dev, stream, false); });
}

int aeon_hip_mask_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
                        const aeon_aug_params* params, const aeon_out_desc* out, void* out_dev,
                        void* stream)
{
    return guarded([&] { return run_batch(ctx, n, descs, src_base, params, out, out_dev, stream, true); });
}

int aeon_hip_augment_pair_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
                                const aeon_img_desc* mask_descs, const void* mask_src_base,
                                const aeon_aug_params* params, const aeon_out_desc* out, void* out_dev,
                                const aeon_out_desc* mask_out, void* mask_out_dev, void* stream)
{
    return guarded([&] {
        if (!ctx || n < 0 || (n > 0 && (!mask_descs || !mask_src_base || !mask_out || !mask_out_dev)))
            fail(AEON_HIP_EINVAL, "null argument");
        if (n == 0) return 0;
        // one launch when every mask is an 8-bit single-channel record without rotation into plain
        // uint8 items (the gather pass the launch's workgroups take after the image tiles); otherwise
        // exactly aeon_hip_augment_batch then aeon_hip_mask_batch
        bool fuse = mask_out->dtype == AEON_DTYPE_U8 && mask_out->channels == 1 && !mask_out->fixed_aspect_ratio &&
                    !mask_out->has_mean && !mask_out->bgr_to_rgb && params;
        for (int i = 0; fuse && i < n; i++)
            fuse = (mask_descs[i].elem_bytes == 0 || mask_descs[i].elem_bytes == 1) && mask_descs[i].channels == 1 &&
                   params[i].angle == 0;
        if (!fuse) {
            run_batch(ctx, n, descs, src_base, params, out, out_dev, stream, false);
            return run_batch(ctx, n, mask_descs, mask_src_base, params, mask_out, mask_out_dev, stream, true);
        }
        const MaskSet ms{mask_descs, mask_src_base, *mask_out, mask_out_dev};
        return run_batch(ctx, n, descs, src_base, params, out, out_dev, stream, false, &ms);
    });
}

int aeon_hip_depthmap_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs, const void* src_base,
                            const aeon_aug_params* params, const aeon_out_desc* out, void* out_dev, void* stream)
{
    return guarded([&] {
        if (out && out->fixed_aspect_ratio)
            fail(AEON_HIP_EINVAL, "depthmap::loader has no fixed_aspect_ratio canvas (etl_depthmap.cpp:98-134)");
        return run_batch(ctx, n, descs, src_base, params, out, out_dev, stream, true);
    });
}

int aeon_hip_release_stream(aeon_hip_ctx* ctx, void* stream)
{
    return guarded([&] {
        if (!ctx) fail(AEON_HIP_EINVAL, "null ctx");
        std::lock_guard<std::mutex> lock(ctx->mu);
        HIP_OK(hipSetDevice(ctx->device));
        // the ring slots of the calls still open on this stream get their completion event now, while
        // the stream exists (the next call on another stream would record it there -- on a destroyed
        // stream by then); the context then holds no reference to the stream
        if (ctx->open_stream == (hipStream_t)stream) {
            close_slots(ctx);
            ctx->open_stream = nullptr;
        }
        return 0;
    });
}

int aeon_hip_synchronize(aeon_hip_ctx* ctx, void* stream)
{
    return guarded([&] {
        if (!ctx) fail(AEON_HIP_EINVAL, "null ctx");
        if (const int rc = aeon_hip_release_stream(ctx, stream)) return rc;
        HIP_OK(hipSetDevice(ctx->device));
        HIP_OK(hipStreamSynchronize((hipStream_t)stream));
        // this stream's word (its calls' kernels are done): read and cleared on the stream itself, the
        // word then handed back (a stream that is reused gets a word again at its next call)
        int32_t* word = stream_error(ctx, (hipStream_t)stream);
        int32_t  err  = 0;
        HIP_OK(hipMemcpyAsync(&err, word, sizeof(err), hipMemcpyDeviceToHost, (hipStream_t)stream));
        if (err != 0) HIP_OK(hipMemsetAsync(word, 0, sizeof(int32_t), (hipStream_t)stream));
        HIP_OK(hipStreamSynchronize((hipStream_t)stream));
        (void)stream_error(ctx, (hipStream_t)stream, true);
        if (err != 0) {
            fail(AEON_HIP_EDEVICE, "device error word " + std::to_string(err) + " (" + device_error_text(err) + ")");
        }
        return 0;
    });
}

int aeon_hip_set_timing(aeon_hip_ctx* ctx, int enable)
{
    return guarded([&] {
        if (!ctx) fail(AEON_HIP_EINVAL, "null ctx");
        std::lock_guard<std::mutex> lock(ctx->mu);
        ctx->timing       = enable > 0;
        ctx->timing_every = std::max(1, enable);
        ctx->timing_calls = 0;
        return 0;
    });
}

int aeon_hip_kernel_times(aeon_hip_ctx* ctx, int kinds, double* ms, double* bytes, long* count)
{
    return guarded([&] {
        if (!ctx || !ms || !bytes || !count) fail(AEON_HIP_EINVAL, "null argument");
        if (kinds < 0) fail(AEON_HIP_EINVAL, "negative kinds");
        std::lock_guard<std::mutex> lock(ctx->mu);
        HIP_OK(hipSetDevice(ctx->device));
        for (KernelTimer& t : ctx->timers) {
            HIP_OK(hipEventSynchronize(t.stop));
            float e = 0;
            HIP_OK(hipEventElapsedTime(&e, t.start, t.stop));
            ctx->ms[t.kind] += e;
            ctx->bytes[t.kind] += t.bytes;
            ctx->count[t.kind] += 1;
            ctx->free_timers.push_back(t);
        }
        ctx->timers.clear();
        for (int k = 0; k < 4; k++) {
            if (k < kinds) ms[k] = ctx->ms[k], bytes[k] = ctx->bytes[k], count[k] = ctx->count[k];
            ctx->ms[k] = ctx->bytes[k] = 0, ctx->count[k] = 0;
        }
        return 0;
    });
}

int aeon_param_factory_create(const char* aug_json, aeon_param_factory** out)
{
    return guarded([&] {
        if (!out) fail(AEON_HIP_EINVAL, "null out");
        Json j = aug_json && *aug_json ? Json::parse(aug_json) : Json();
        *out   = new aeon_param_factory(j);
        return 0;
    });
}

int aeon_param_factory_destroy(aeon_param_factory* f)
{
    delete f;
    return 0;
}

int aeon_make_params(aeon_param_factory* f, uint32_t* state, int in_w, int in_h, int out_w, int out_h,
                     aeon_aug_params* out)
{
    return guarded([&] {
        if (!f || !state || !out) fail(AEON_HIP_EINVAL, "null argument");
        std::lock_guard<std::mutex> lock(f->mu);
        TrackedEngine eng(*state);
        f->f.make_params(eng, in_w, in_h, out_w, out_h, out);
        *state = eng.last;
        return 0;
    });
}

int aeon_make_ssd_params(aeon_param_factory* f, uint32_t* state, int in_w, int in_h, int out_w, int out_h,
                         const float* boxes, int n_boxes, aeon_aug_params* out)
{
    return guarded([&] {
        if (!f || !state || !out || n_boxes < 0 || (n_boxes > 0 && !boxes)) fail(AEON_HIP_EINVAL, "null argument");
        std::lock_guard<std::mutex> lock(f->mu);
        TrackedEngine eng(*state);
        f->f.make_ssd_params(eng, in_w, in_h, out_w, out_h, boxes, n_boxes, out);
        *state = eng.last;
        return 0;
    });
}

int aeon_png_info(const void* data, size_t size, int* width, int* height, int* bit_depth, int* color_type)
{
    return guarded([&] {
        if (!data || !width || !height || !bit_depth || !color_type) fail(AEON_HIP_EINVAL, "null argument");
        png_header(data, size, width, height, bit_depth, color_type);
        return 0;
    });
}

int aeon_decode_png(const void* data, size_t size, int mode, void* dst, size_t stride, int* elem_bytes)
{
    return guarded([&] {
        if (!data || !dst) fail(AEON_HIP_EINVAL, "null argument");
        if (mode < AEON_PNG_BGR8 || mode > AEON_PNG_ANYDEPTH) fail(AEON_HIP_EINVAL, "unknown PNG decode mode");
        int w, h, depth, ctype;
        png_header(data, size, &w, &h, &depth, &ctype);
        const size_t eb = (mode == AEON_PNG_ANYDEPTH && depth == 16 && ctype != 3) ? 2 : 1;
        if (stride < (size_t)w * (mode == AEON_PNG_BGR8 ? 3 : 1) * eb) fail(AEON_HIP_EINVAL, "stride too small");
        png_decode(data, size, mode, dst, stride, elem_bytes);
        return 0;
    });
}

int aeon_batch_sample_patches(aeon_param_factory* f, int sampler, uint32_t* state, const float* nboxes, int n,
                              float* out, int cap, int* n_out)
{
    return guarded([&] {
        if (!f || !state || !n_out || n < 0 || (n > 0 && !nboxes) || cap < 0 || (cap > 0 && !out))
            fail(AEON_HIP_EINVAL, "null argument");
        std::lock_guard<std::mutex> lock(f->mu);
        if (sampler < 0 || sampler >= (int)f->f.batch_samplers.size()) fail(AEON_HIP_EINVAL, "sampler index out of range");
        TrackedEngine     eng(*state);
        std::vector<nbox> objects, samples;
        for (int i = 0; i < n; i++)
            objects.emplace_back(nboxes[4 * i], nboxes[4 * i + 1], nboxes[4 * i + 2], nboxes[4 * i + 3]);
        f->f.batch_samplers[sampler].sample_patches(eng, objects, samples);
        *n_out = (int)samples.size();
        for (int i = 0; i < (int)samples.size() && i < cap; i++) {
            out[4 * i] = samples[i].xmin, out[4 * i + 1] = samples[i].ymin;
            out[4 * i + 2] = samples[i].xmax, out[4 * i + 3] = samples[i].ymax;
        }
        *state = eng.last;
        return 0;
    });
}

int aeon_seed_slots(uint32_t seed, int n, uint32_t* states)
{
    return guarded([&] {
        if (n < 0 || (n > 0 && !states)) fail(AEON_HIP_EINVAL, "bad arguments");
        std::minstd_rand0 g(seed);
        for (int i = 0; i < n; i++) {
            uint32_t s = g() % 2147483647u;
            states[i]  = s == 0 ? 1 : s;
        }
        return 0;
    });
}

int aeon_jpeg_info(const void* data, size_t size, int* width, int* height, int* components)
{
    return guarded([&] {
        if (!data || !width || !height || !components) fail(AEON_HIP_EINVAL, "null argument");
        jpeg_info(data, size, width, height, components);
        return 0;
    });
}

int aeon_jpeg_entropy_decode(const void* data, size_t size, int* width, int* height, int* components,
                             int64_t* n_blocks, int64_t* n_values, uint64_t* hash)
{
    return guarded([&] {
        if (!data || !width || !height || !components || !n_blocks || !n_values || !hash)
            fail(AEON_HIP_EINVAL, "null argument");
        jpeg_entropy_only(data, size, width, height, components, n_blocks, n_values, hash);
        return 0;
    });
}

int aeon_jpeg_host_stage(const void* data, size_t size, int* gpu_entropy, int64_t* staged_bytes)
{
    return guarded([&] {
        if (!data || !gpu_entropy || !staged_bytes) fail(AEON_HIP_EINVAL, "null argument");
        jpeg_host_stage(data, size, gpu_entropy, staged_bytes);
        return 0;
    });
}

int aeon_hip_decode_jpeg_batch(aeon_hip_ctx* ctx, int n, const void* const* data, const size_t* sizes,
                               const aeon_img_desc* descs, void* dst_base, void* stream)
{
    return guarded([&] {
        if (!ctx || n < 0 || (n > 0 && (!data || !sizes || !descs || !dst_base))) fail(AEON_HIP_EINVAL, "null argument");
        if (n == 0) return 0;
        HIP_OK(hipSetDevice(ctx->device));
        if (!ctx->jpeg) ctx->jpeg = jpeg_state_create(ctx->host_pool, ctx->jpeg_gpu_huff);
        KernelTimer t{};
        bool        timed = false;
        if (ctx->timing) {
            std::lock_guard<std::mutex> lock(ctx->mu);
            timed = (ctx->timing_calls++ % ctx->timing_every) == ctx->timing_every - 1;
            if (timed) {
                double px = 0;
                for (int i = 0; i < n; i++) px += (double)descs[i].width * descs[i].height * descs[i].channels;
                t = take_timer(ctx, kTimerJpeg, px);
            }
        }
        jpeg_decode_batch(ctx->jpeg, n, data, sizes, descs, dst_base, stream_error(ctx, (hipStream_t)stream), (hipStream_t)stream,
                          timed ? t.start : nullptr,
                          timed ? t.stop : nullptr);
        if (timed) {
            std::lock_guard<std::mutex> lock(ctx->mu);
            ctx->timers.push_back(t);
        }
        return 0;
    });
}

int aeon_unbiased_round(float x, int64_t* out)
{
    return guarded([&] {
        if (!out) fail(AEON_HIP_EINVAL, "null out");
        *out = unbiased_round(x);
        return 0;
    });
}

int aeon_calculate_scale(int width, int height, int output_width, int output_height, float* scale)
{
    return guarded([&] {
        if (!scale) fail(AEON_HIP_EINVAL, "null out");
        *scale = calculate_scale(width, height, output_width, output_height);
        return 0;
    });
}

int aeon_cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* res_w, float* res_h)
{
    return guarded([&] {
        if (!res_w || !res_h) fail(AEON_HIP_EINVAL, "null out");
        cropbox_max_proportional(in_w, in_h, out_w, out_h, res_w, res_h);
        return 0;
    });
}

int aeon_hip_host_alloc(size_t bytes, void** out)
{
    return guarded([&] {
        if (!out) fail(AEON_HIP_EINVAL, "null out");
        HIP_OK(hipHostMalloc(out, bytes, hipHostMallocDefault));
        return 0;
    });
}

int aeon_hip_host_free(void* p)
{
    return guarded([&] {
        if (p) HIP_OK(hipHostFree(p));
        return 0;
    });
}

const char* aeon_hip_last_error(void) { return g_err.c_str(); }
int aeon_hip_debug_uncached_blocks(uint64_t* ranges, int cap, int* n)
{
    return guarded([&] {
        if (!n || (cap > 0 && !ranges)) fail(AEON_HIP_EINVAL, "null argument");
        std::lock_guard<std::mutex> lock(g_vram_pool_mu);
        *n = (int)g_vram_all.size();
        for (int i = 0; i < cap && i < *n; i++) {
            ranges[2 * i]     = (uint64_t)(uintptr_t)g_vram_all[i].first;
            ranges[2 * i + 1] = (uint64_t)(uintptr_t)g_vram_all[i].first + g_vram_all[i].second;
        }
        return 0;
    });
}

const char* aeon_hip_version(void) { return "aeon-hip 0.1 (gfx950)"; }

} // extern "C"
