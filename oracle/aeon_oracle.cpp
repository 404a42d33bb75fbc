// aeon_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see aeon_oracle.h).
//
// A from-scratch CPU restatement of aeon's image path with the OpenCV-2.4 (SSE2 build)
// arithmetic it inherits.  Every function names the reference code it restates.
// Built with -ffp-contract=off so float expressions round exactly like the x86 SSE2
// reference build (no FMA contraction).
#include "aeon_oracle.h"

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>

#include <pthread.h>
#include <sched.h>
#include <vector>

namespace {

thread_local std::string g_err;

// ---- OpenCV scalar helpers (x86-64 SSE2: cvRound = cvtsd2si, round-half-even) ----------
inline int cv_round(double v) { return (int)std::nearbyint(v); }
inline int cv_roundf(float v) { return (int)std::nearbyintf(v); }
inline int cv_floor(double v) { return (int)std::floor(v); }
inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }
inline int sat_s16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
inline uint8_t sat_u8f(float v) { return sat_u8(cv_roundf(v)); }

// A minstd_rand0 wrapper whose state word can be read back (the LCG state == last output).
struct Engine {
    using result_type = std::minstd_rand0::result_type;
    std::minstd_rand0 e;
    result_type       last;
    static constexpr result_type min() { return std::minstd_rand0::min(); }
    static constexpr result_type max() { return std::minstd_rand0::max(); }
    explicit Engine(uint32_t s) : e(s), last(s) {}
    result_type operator()() { return last = e(); }
};

// ---- augment::image::param_factory (src/augment_image.cpp:28-89, .hpp:141-204) --------------
struct Factory {
    orc_aug_config                        c;
    std::uniform_real_distribution<float> scale, hdist, contrast, brightness, saturation;
    std::uniform_real_distribution<float> crop_offset{0.5f, 0.5f};
    std::uniform_int_distribution<int>    angle, hue;
    std::uniform_int_distribution<int>    pad_offset{0, 0};
    std::normal_distribution<float>       lighting;
    std::bernoulli_distribution           flip{0};

    explicit Factory(const orc_aug_config& cfg)
        : c(cfg)
        , scale{cfg.scale_min, cfg.scale_max}
        , hdist{cfg.hdist_min, cfg.hdist_max}
        , contrast{cfg.contrast_min, cfg.contrast_max}
        , brightness{cfg.brightness_min, cfg.brightness_max}
        , saturation{cfg.saturation_min, cfg.saturation_max}
        , angle{cfg.angle_min, cfg.angle_max}
        , hue{cfg.hue_min, cfg.hue_max}
        , lighting{cfg.lighting_mean, cfg.lighting_stddev}
    {
        if (cfg.flip_enable) flip = std::bernoulli_distribution{0.5};
        if (!cfg.center) crop_offset = std::uniform_real_distribution<float>{0.0f, 1.0f};
        if (cfg.padding > 0) pad_offset = std::uniform_int_distribution<int>(0, cfg.padding * 2);
    }
};

// src/util.cpp:212-239
int unbiased_round(float x)
{
    float i;
    float frac = std::modf(x, &i);
    int   ip   = int(i);
    int   rc;
    if (std::fabs(frac) == 0.5f) {
        if (ip % 2 == 0) rc = ip;
        else {
            rc = std::fabs(x) + 0.5;
            rc = x < 0.0 ? -rc : rc;
        }
    } else {
        rc = std::floor(std::fabs(x) + 0.5);
        rc = x < 0.0 ? -rc : rc;
    }
    return rc;
}

// image.cpp:108-116 get_resized_short_size
void resized_short_size(int in_w, int in_h, int target, int* ow, int* oh)
{
    float pct = static_cast<float>(target) / (float)std::min(in_h, in_w);
    *ow = static_cast<int>(std::round((float)in_w * pct));
    *oh = static_cast<int>(std::round((float)in_h * pct));
}

// image.cpp:214-224 calculate_scale (cv::Size int input)
float calculate_scale(int w, int h, int ow, int oh)
{
    float im_scale = (float)ow / (float)w;
    float rh       = (float)h * im_scale;
    if (rh > oh) im_scale = (float)oh / (float)h;
    return im_scale;
}

// image.cpp:226-237 cropbox_max_proportional
void cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* rw, float* rh)
{
    float w = out_w, h = out_h;
    float s = in_w / w;
    w *= s;
    h *= s;
    if (h > in_h) {
        s = in_h / h;
        w *= s;
        h *= s;
    }
    *rw = w;
    *rh = h;
}

// param_factory::make_params (src/augment_image.cpp:107-230)
void make_params(const Factory& fc, Engine& eng, int in_w, int in_h, int out_w, int out_h,
                 orc_params* p)
{
    Factory&              f = const_cast<Factory&>(fc); // distributions are `mutable` in aeon
    const orc_aug_config& c = f.c;
    std::memset(p, 0, sizeof(*p));
    p->expand_ratio = 1.0f; // augment::image::params default (augment_image.hpp:99)
    p->out_w      = out_w;
    p->out_h      = out_h;
    p->angle      = f.angle(eng);
    p->flip       = f.flip(eng) ? 1 : 0;
    p->hue        = f.hue(eng);
    p->contrast   = f.contrast(eng);
    p->brightness = f.brightness(eng);
    p->saturation = f.saturation(eng);
    p->padding    = c.padding;
    p->resize_short_size = c.resize_short_size;
    p->interp            = c.interp;

    float in_sw = (float)in_w, in_sh = (float)in_h; // cv::Size2f input_size

    if (!c.crop_enable) {
        int ox       = f.pad_offset(eng);
        int oy       = f.pad_offset(eng);
        p->pad_off_x = ox;
        p->pad_off_y = oy;
        p->crop_x = 0;
        p->crop_y = 0;
        p->crop_w = cv_roundf(in_sw);
        p->crop_h = cv_roundf(in_sh);
        float s   = c.fixed_scaling_factor > 0 ? c.fixed_scaling_factor
                                               : calculate_scale(in_w, in_h, out_w, out_h);
        in_sw *= s;
        in_sh *= s;
        p->out_w = unbiased_round(in_sw);
        p->out_h = unbiased_round(in_sh);
    } else if (c.do_area_scale) {
        float hd = f.hdist(eng);
        hd       = std::sqrt(hd);
        float sw = hd, sh = 1 / hd;
        float bound = std::min((float)in_w / (float)in_h / (sw * sw),
                               (float)in_h / (float)in_w / (sh * sh));
        float smax = std::min(f.scale.max(), bound);
        float smin = std::min(f.scale.min(), bound);
        std::uniform_real_distribution<float> scale2{smin, smax};
        float target_area = std::sqrt((float)((size_t)in_h * (size_t)in_w) * scale2(eng));
        sw *= target_area;
        sh *= target_area;
        float offx = f.crop_offset(eng);
        float offy = f.crop_offset(eng);
        p->crop_x  = (int)((in_sw - sw) * offx);
        p->crop_y  = (int)((in_sh - sh) * offy);
        p->crop_w  = cv_roundf(sw);
        p->crop_h  = cv_roundf(sh);
    } else {
        if (c.padding > 0) {
            throw std::invalid_argument("crop_enable should not be true: when padding is defined");
        }
        float image_scale = f.scale(eng);
        float hd          = f.hdist(eng);
        float osw = (float)out_w * hd, osh = (float)out_h;
        if (c.resize_short_size > 0) {
            int rw, rh;
            resized_short_size(in_w, in_h, c.resize_short_size, &rw, &rh);
            in_sw = (float)rw;
            in_sh = (float)rh;
        }
        float cw, ch;
        cropbox_max_proportional(in_sw, in_sh, osw, osh, &cw, &ch);
        cw *= image_scale; // cropbox_linear_scale (image.cpp:239-242)
        ch *= image_scale;
        float offx = f.crop_offset(eng);
        float offy = f.crop_offset(eng);
        p->crop_x  = (int)((in_sw - cw) * offx); // cropbox_shift truncates (image.cpp:263-273)
        p->crop_y  = (int)((in_sh - ch) * offy);
        p->crop_w  = cv_roundf(cw);             // cv::Rect(Point2i, Size2f): saturate_cast
        p->crop_h  = cv_roundf(ch);
    }

    if (f.lighting.stddev() != 0) {
        for (int i = 0; i < 3; i++) p->lighting[i] = f.lighting(eng);
        p->n_lighting      = 3;
        p->color_noise_std = f.lighting.stddev();
    }
}

// ---- make_ssd_params (src/augment_image.cpp:232-586, normalized_box.cpp, boundingbox.cpp) ------
// normalized_box::box: constructor rejects coordinates outside [0, 1] +- nervana::epsilon
struct NBox {
    float x0, y0, x1, y1;
};
NBox make_nbox(float x0, float y0, float x1, float y1)
{
    const float e  = 0.00001f;
    auto        ok = [&](float v) { return v >= 0.0f - e && v <= 1.0f + e; };
    if (!(ok(x0) && ok(x1) && ok(y0) && ok(y1))) throw std::invalid_argument("bounding box is not properly normalized");
    return NBox{x0, y0, x1, y1};
}
float nbox_size(const NBox& b) { return (b.x1 < b.x0 || b.y1 < b.y0) ? 0.0f : (b.x1 - b.x0) * (b.y1 - b.y0); }
NBox  nbox_intersect(const NBox& a, const NBox& b)
{
    if (b.x0 > a.x1 || b.x1 < a.x0 || b.y0 > a.y1 || b.y1 < a.y0) return NBox{0, 0, 0, 0};
    return make_nbox(std::max(a.x0, b.x0), std::max(a.y0, b.y0), std::min(a.x1, b.x1), std::min(a.y1, b.y1));
}
float jaccard(const NBox& a, const NBox& b)
{
    float i = nbox_size(nbox_intersect(a, b));
    return i == 0.f ? 0.f : i / (nbox_size(a) + nbox_size(b) - i);
}
float coverage_of(const NBox& own, const NBox& other)
{
    float i = nbox_size(nbox_intersect(own, other));
    return i > 0 ? i / nbox_size(own) : 0.f;
}
bool satisfies(const orc_batch_sampler& bs, const NBox& s, const std::vector<NBox>& objs)
{
    auto       has = [](float v) { return v == v; };
    const bool jac = has(bs.min_jaccard) || has(bs.max_jaccard);
    const bool sc  = has(bs.min_sample_cov) || has(bs.max_sample_cov);
    const bool oc  = has(bs.min_object_cov) || has(bs.max_object_cov);
    if (!jac && !sc && !oc) return true;
    bool found = false; // not reset per object: a partial pass on one object carries over
    for (const NBox& o : objs) {
        if (jac) {
            float v = jaccard(s, o);
            if ((has(bs.min_jaccard) && v < bs.min_jaccard) || (has(bs.max_jaccard) && v > bs.max_jaccard)) continue;
            found = true;
        }
        if (sc) {
            float v = coverage_of(s, o);
            if ((has(bs.min_sample_cov) && v < bs.min_sample_cov) || (has(bs.max_sample_cov) && v > bs.max_sample_cov))
                continue;
            found = true;
        }
        if (oc) {
            float v = coverage_of(o, s);
            if ((has(bs.min_object_cov) && v < bs.min_object_cov) || (has(bs.max_object_cov) && v > bs.max_object_cov))
                continue;
            found = true;
        }
        if (found) return true;
    }
    return found;
}

// ---- a light u8 image view ------------------------------------------------------------------
struct Img {
    int                  w = 0, h = 0, cn = 0, stride = 0;
    const uint8_t*       data = nullptr;
    std::vector<uint8_t> own;
    uint8_t*       row(int y) { return const_cast<uint8_t*>(data) + (size_t)y * stride; }
    const uint8_t* row(int y) const { return data + (size_t)y * stride; }
    static Img alloc(int w, int h, int cn)
    {
        Img r;
        r.w = w, r.h = h, r.cn = cn, r.stride = w * cn;
        r.own.assign((size_t)w * h * cn, 0);
        r.data = r.own.data();
        return r;
    }
    static Img view(const uint8_t* d, int w, int h, int cn, int stride)
    {
        Img r;
        r.w = w, r.h = h, r.cn = cn, r.stride = stride, r.data = d;
        return r;
    }
    Img clone() const
    {
        Img r = alloc(w, h, cn);
        for (int y = 0; y < h; y++) std::memcpy(r.row(y), row(y), (size_t)w * cn);
        return r;
    }
};

// ---- cv::resize INTER_LINEAR, 8U (OpenCV 2.4 imgwarp.cpp resize / resizeGeneric_ /
//      HResizeLinear / VResizeLinear + VResizeLinearVec_32s8u, ResizeAreaFastVec) ----------------
void resize_linear(const Img& s, Img& d)
{
    const int sw = s.w, sh = s.h, cn = s.cn, dw = d.w, dh = d.h;
    if (sw == dw && sh == dh) {
        for (int y = 0; y < sh; y++) std::memcpy(d.row(y), s.row(y), (size_t)sw * cn);
        return;
    }
    double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    int    isx = cv_round(scale_x), isy = cv_round(scale_y);
    bool   area_fast = std::abs(scale_x - isx) < DBL_EPSILON && std::abs(scale_y - isy) < DBL_EPSILON;
    if (area_fast && isx == 2 && isy == 2 && (cn == 1 || cn == 3 || cn == 4)) {
        // INTER_LINEAR at exactly 2x is routed to INTER_AREA's fast path (resizeAreaFast_).
        for (int dy = 0; dy < dh; dy++) {
            const uint8_t* S0 = s.row(2 * dy);
            const uint8_t* S1 = s.row(2 * dy + 1);
            uint8_t*       D  = d.row(dy);
            for (int dx = 0; dx < dw * cn; dx++) {
                int px = dx / cn, k = dx % cn, i = px * 2 * cn + k;
                D[dx]  = (uint8_t)((S0[i] + S0[i + cn] + S1[i] + S1[i + cn] + 2) >> 2);
            }
        }
        return;
    }

    const int        W = dw * cn;
    std::vector<int> xofs(W), a0(W), a1(W);
    int              xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int   sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        int c0 = sat_s16(cv_roundf((1.f - fx) * 2048)), c1 = sat_s16(cv_roundf(fx * 2048));
        for (int k = 0; k < cn; k++) {
            xofs[dx * cn + k] = sx * cn + k;
            a0[dx * cn + k]   = c0;
            a1[dx * cn + k]   = c1;
        }
    }
    const int xmax_e = xmax * cn;
    // SIMD / scalar split of VResizeLinearVec_32s8u: 16-wide while x <= W-16, then 4-wide
    // while x < W-4; the remaining elements use the scalar FixedPtCast formula.
    int xv = 0;
    if (W >= 16) xv = (W / 16) * 16;
    while (xv < W - 4) xv += 4;

    std::vector<int> H0(W), H1(W);
    auto hrow = [&](const uint8_t* S, std::vector<int>& H) {
        for (int x = 0; x < W; x++) {
            int sx = xofs[x];
            H[x]   = x < xmax_e ? S[sx] * a0[x] + S[sx + cn] * a1[x] : S[sx] * 2048;
        }
    };
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int   sy = cv_floor(fy);
        fy -= sy;
        int b0 = sat_s16(cv_roundf((1.f - fy) * 2048)), b1 = sat_s16(cv_roundf(fy * 2048));
        int r0 = std::min(std::max(sy, 0), sh - 1), r1 = std::min(std::max(sy + 1, 0), sh - 1);
        hrow(s.row(r0), H0);
        hrow(s.row(r1), H1);
        uint8_t* D = d.row(dy);
        for (int x = 0; x < W; x++) {
            if (x < xv) {
                int h0 = sat_s16(H0[x] >> 4), h1 = sat_s16(H1[x] >> 4);
                int m  = sat_s16(((h0 * (int)(short)b0) >> 16) + ((h1 * (int)(short)b1) >> 16));
                int v  = sat_s16(m + 2) >> 2;
                D[x]   = sat_u8(v);
            } else {
                D[x] = sat_u8((H0[x] * b0 + H1[x] * b1 + (1 << 21)) >> 22);
            }
        }
    }
}

// cv::resize INTER_NEAREST (resizeNN)
void resize_nearest(const Img& s, Img& d)
{
    double fx = (double)d.w / s.w, fy = (double)d.h / s.h;
    double ifx = 1. / fx, ify = 1. / fy;
    for (int y = 0; y < d.h; y++) {
        int            sy = std::min(cv_floor(y * ify), s.h - 1);
        const uint8_t* S  = s.row(sy);
        uint8_t*       D  = d.row(y);
        for (int x = 0; x < d.w; x++) {
            int sx = std::min(cv_floor(x * ifx), s.w - 1);
            for (int k = 0; k < s.cn; k++) D[x * s.cn + k] = S[sx * s.cn + k];
        }
    }
}


// ---- cv::resize INTER_CUBIC / INTER_LANCZOS4 / INTER_AREA, 8U --------------------------------
// PARITY UNPINNED: aeon's tests hold no output of these methods (its interpolation_method map,
// src/image.cpp:30-36, reaches them from the "interpolation_method" config, used by image::resize
// :93-106 and image::resize_short :118-127).  Restated from OpenCV 2.4.9 imgwarp.cpp: cv::resize's
// coefficient set-up (x: sx/fx with the xmin/xmax clamps, y: unclamped sy, rows clipped),
// interpolateCubic (A = -0.75) / interpolateLanczos4, 11-bit fixed-point coefficients
// (saturate_cast<short>(c * 2048)), resizeGeneric_ with HResizeCubic / HResizeLanczos4 (exact int,
// edge taps clamped) and VResizeCubic (VResizeCubicVec_32s8u, SSE2: float sums, 8 elements at a time
// while x <= W - 8, cvtps round-half-even, packs/packus saturation; the scalar tail
// FixedPtCast<int, uchar, 22>) / VResizeLanczos4 (all scalar FixedPtCast, int32 sums wrapping as on
// x86); INTER_AREA: downscale in both axes -> resizeAreaFast_ for integer factors (2x2: the
// (a+b+c+d+2)>>2 fast mode; otherwise saturate_cast<uchar>(sum * (1.f/area))) or resizeArea_ with
// computeResizeAreaTab (float sums in table order); otherwise bilinear with area-mode coefficients.
enum { ORC_LINEAR = 0, ORC_NEAREST = 1, ORC_CUBIC = 2, ORC_AREA = 3, ORC_LANCZOS4 = 4 };

static void interpolate_cubic(float x, float* c)
{
    const float A = -0.75f;
    c[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
    c[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
    c[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
    c[3] = 1.f - c[0] - c[1] - c[2];
}

void interpolate_lanczos4(float x, float* c)
{
    static const double s45   = 0.70710678118654752440084436210485;
    static const double cs[][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
    const double        kPi   = 3.1415926535897932384626433832795;
    if (x < FLT_EPSILON) {
        for (int i = 0; i < 8; i++) c[i] = 0;
        c[3] = 1;
        return;
    }
    float  sum = 0;
    double y0 = -(x + 3) * kPi * 0.25, s0 = std::sin(y0), c0 = std::cos(y0);
    for (int i = 0; i < 8; i++) {
        double y = -(x + 3 - i) * kPi * 0.25;
        c[i]     = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
        sum += c[i];
    }
    sum = 1.f / sum;
    for (int i = 0; i < 8; i++) c[i] *= sum;
}

// cv::resize's coefficient set-up for the ksize-tap filters (ksize 2 with area_mode: INTER_AREA's
// bilinear emulation): per destination column its (clamped) sx and fixed-point taps, per row sy.
struct GenTaps {
    std::vector<int> sx, sy;       // first-tap anchors (x after the clamps; y raw)
    std::vector<short> ax, by;     // ksize coefficients per column / row
};
static void coeffs_for(int interp, float f, float* c)
{
    if (interp == ORC_CUBIC) interpolate_cubic(f, c);
    else if (interp == ORC_LANCZOS4) interpolate_lanczos4(f, c);
    else c[0] = 1.f - f, c[1] = f;
}
static GenTaps gen_taps(int interp, int ksize, bool area_mode, int sw, int sh, int dw, int dh)
{
    GenTaps T;
    const double inv_sx = (double)dw / sw, inv_sy = (double)dh / sh;
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    const int    k2 = ksize / 2;
    T.sx.resize(dw), T.sy.resize(dh), T.ax.resize((size_t)dw * ksize), T.by.resize((size_t)dh * ksize);
    float cbuf[8];
    for (int dx = 0; dx < dw; dx++) {
        float fx;
        int   sx;
        if (!area_mode) {
            fx = (float)((dx + 0.5) * scale_x - 0.5);
            sx = cv_floor(fx);
            fx -= sx;
        } else {
            sx = cv_floor(dx * scale_x);
            fx = (float)((dx + 1) - (sx + 1) * inv_sx);
            fx = fx <= 0 ? 0.f : fx - cv_floor(fx);
        }
        if (sx < k2 - 1 && sx < 0) fx = 0, sx = 0;
        if (sx + k2 >= sw && sx >= sw - 1) fx = 0, sx = sw - 1;
        T.sx[dx] = sx;
        coeffs_for(interp, fx, cbuf);
        for (int k = 0; k < ksize; k++) T.ax[(size_t)dx * ksize + k] = (short)sat_s16(cv_roundf(cbuf[k] * 2048));
    }
    for (int dy = 0; dy < dh; dy++) {
        float fy;
        int   sy;
        if (!area_mode) {
            fy = (float)((dy + 0.5) * scale_y - 0.5);
            sy = cv_floor(fy);
            fy -= sy;
        } else {
            sy = cv_floor(dy * scale_y);
            fy = (float)((dy + 1) - (sy + 1) * inv_sy);
            fy = fy <= 0 ? 0.f : fy - cv_floor(fy);
        }
        T.sy[dy] = sy;
        coeffs_for(interp, fy, cbuf);
        for (int k = 0; k < ksize; k++) T.by[(size_t)dy * ksize + k] = (short)sat_s16(cv_roundf(cbuf[k] * 2048));
    }
    return T;
}

// First element of a W-element row on the scalar tail of the ksize-tap vertical pass (SSE2 build):
// linear VResizeLinearVec_32s8u (16 then 4 at a time), cubic VResizeCubicVec_32s8u (8 at a time),
// Lanczos4 none.
int vresize_simd_end(int ksize, int W)
{
    int x = 0;
    if (ksize == 2) {
        x = W >= 16 ? (W / 16) * 16 : 0;
        while (x < W - 4) x += 4;
    } else if (ksize == 4) {
        while (x <= W - 8) x += 8;
    }
    return x;
}

// resizeGeneric_ for ksize 2 (area-mode bilinear), 4 (cubic) and 8 (Lanczos4), 8U.
void resize_generic(const Img& s, Img& d, int interp, bool area_mode)
{
    const int ksize = interp == ORC_CUBIC ? 4 : (interp == ORC_LANCZOS4 ? 8 : 2), k2 = ksize / 2;
    const int sw = s.w, sh = s.h, cn = s.cn, dw = d.w, dh = d.h, W = dw * cn;
    const GenTaps T = gen_taps(interp, ksize, area_mode, sw, sh, dw, dh);
    const int xv = vresize_simd_end(ksize, W);
    std::vector<int> H((size_t)ksize * W);
    for (int dy = 0; dy < dh; dy++) {
        // horizontal pass of the ksize source rows (clip(sy - k2 + 1 + k, 0, sh))
        for (int k = 0; k < ksize; k++) {
            const int      r = std::min(std::max(T.sy[dy] - k2 + 1 + k, 0), sh - 1);
            const uint8_t* S = s.row(r);
            for (int dx = 0; dx < dw; dx++)
                for (int c = 0; c < cn; c++) {
                    int v = 0;
                    for (int j = 0; j < ksize; j++) {
                        const int x = std::min(std::max(T.sx[dx] - k2 + 1 + j, 0), sw - 1);
                        v += S[x * cn + c] * T.ax[(size_t)dx * ksize + j];
                    }
                    H[(size_t)k * W + dx * cn + c] = v;
                }
        }
        const short* b = &T.by[(size_t)dy * ksize];
        uint8_t*     D = d.row(dy);
        for (int x = 0; x < W; x++) {
            if (x < xv && ksize == 2) { // VResizeLinearVec_32s8u
                int h0 = sat_s16(H[x] >> 4), h1 = sat_s16(H[W + x] >> 4);
                int m  = sat_s16(((h0 * (int)b[0]) >> 16) + ((h1 * (int)b[1]) >> 16));
                D[x]   = sat_u8(sat_s16(m + 2) >> 2);
            } else if (x < xv && ksize == 4) { // VResizeCubicVec_32s8u: float, in SSE's order
                const float sc = 1.f / (2048 * 2048);
                float       v  = (float)H[x] * ((float)b[0] * sc) + (float)H[W + x] * ((float)b[1] * sc);
                v              = v + (float)H[2 * W + x] * ((float)b[2] * sc);
                v              = v + (float)H[3 * W + x] * ((float)b[3] * sc);
                D[x]           = sat_u8(sat_s16(cv_roundf(v)));
            } else { // FixedPtCast<int, uchar, 22> over int sums (wrapping as x86 int arithmetic)
                uint32_t acc = 0;
                for (int k = 0; k < ksize; k++) acc += (uint32_t)H[(size_t)k * W + x] * (uint32_t)(int)b[k];
                D[x] = sat_u8((int32_t)(acc + (1u << 21)) >> 22);
            }
        }
    }
}

// resizeAreaFast_ (integer factors iscale_x x iscale_y, both >= 1), 8U.
void resize_area_fast(const Img& s, Img& d, int isx, int isy)
{
    const int cn = s.cn;
    const bool fast2 = isx == 2 && isy == 2 && (cn == 1 || cn == 3 || cn == 4);
    const float scale = 1.f / (isx * isy);
    for (int dy = 0; dy < d.h; dy++) {
        uint8_t* D = d.row(dy);
        for (int dx = 0; dx < d.w; dx++)
            for (int c = 0; c < cn; c++) {
                int sum = 0;
                for (int y = 0; y < isy; y++)
                    for (int x = 0; x < isx; x++) sum += s.row(dy * isy + y)[(dx * isx + x) * cn + c];
                D[dx * cn + c] = fast2 ? (uint8_t)((sum + 2) >> 2) : sat_u8(cv_roundf((float)sum * scale));
            }
    }
}

// computeResizeAreaTab + resizeArea_ (non-integer downscale in both axes), 8U.
struct AreaTab {
    int   di, si;
    float alpha;
};
std::vector<AreaTab> area_tab(int ssize, int dsize, double scale)
{
    std::vector<AreaTab> tab;
    for (int dx = 0; dx < dsize; dx++) {
        const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
        const double cell = std::min(scale, ssize - fsx1);
        int          sx1 = (int)std::ceil(fsx1), sx2 = cv_floor(fsx2);
        sx2 = std::min(sx2, ssize - 1);
        sx1 = std::min(sx1, sx2);
        if (sx1 - fsx1 > 1e-3) tab.push_back({dx, sx1 - 1, (float)((sx1 - fsx1) / cell)});
        for (int sx = sx1; sx < sx2; sx++) tab.push_back({dx, sx, (float)(1.0 / cell)});
        if (fsx2 - sx2 > 1e-3) tab.push_back({dx, sx2, (float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell)});
    }
    return tab;
}
void resize_area_generic(const Img& s, Img& d, double scale_x, double scale_y)
{
    const int cn = s.cn;
    const std::vector<AreaTab> xt = area_tab(s.w, d.w, scale_x), yt = area_tab(s.h, d.h, scale_y);
    std::vector<float> buf((size_t)d.w * cn), sum((size_t)d.w * cn, 0.f);
    int prev = yt.empty() ? 0 : yt[0].di;
    for (const AreaTab& y : yt) {
        std::fill(buf.begin(), buf.end(), 0.f);
        const uint8_t* S = s.row(y.si);
        for (const AreaTab& x : xt)
            for (int c = 0; c < cn; c++) buf[(size_t)x.di * cn + c] = buf[(size_t)x.di * cn + c] + S[x.si * cn + c] * x.alpha;
        if (y.di != prev) {
            uint8_t* D = d.row(prev);
            for (size_t i = 0; i < buf.size(); i++) D[i] = sat_u8f(sum[i]), sum[i] = y.alpha * buf[i];
            prev = y.di;
        } else {
            for (size_t i = 0; i < buf.size(); i++) sum[i] = sum[i] + y.alpha * buf[i];
        }
    }
    uint8_t* D = d.row(prev);
    for (size_t i = 0; i < sum.size(); i++) D[i] = sat_u8f(sum[i]);
}

// cv::resize (OpenCV 2.4.9) for every interpolation aeon's config names, 8U.
void resize_cv(const Img& s, Img& d, int interp)
{
    if (interp == ORC_NEAREST) return resize_nearest(s, d);
    if (interp == ORC_LINEAR) return resize_linear(s, d);
    const double inv_sx = (double)d.w / s.w, inv_sy = (double)d.h / s.h;
    const double scale_x = 1. / inv_sx, scale_y = 1. / inv_sy;
    if (interp == ORC_AREA && scale_x >= 1 && scale_y >= 1) {
        const int isx = cv_round(scale_x), isy = cv_round(scale_y);
        if (std::abs(scale_x - isx) < DBL_EPSILON && std::abs(scale_y - isy) < DBL_EPSILON)
            return resize_area_fast(s, d, isx, isy);
        return resize_area_generic(s, d, scale_x, scale_y);
    }
    resize_generic(s, d, interp == ORC_AREA ? ORC_LINEAR : interp, interp == ORC_AREA);
}

// image::resize (image.cpp:93-106): identity when the size already matches.
void resize_any(const Img& s, Img& d, int interp)
{
    if (s.w == d.w && s.h == d.h) {
        for (int y = 0; y < s.h; y++) std::memcpy(d.row(y), s.row(y), (size_t)s.w * s.cn);
        return;
    }
    resize_cv(s, d, interp);
}

// ---- photometric::cbsjitter (src/image.cpp:358-406) -----------------------------------------
void bs_transform(Img& m, float brightness, float saturation)
{
    // satmtx = brightness * (saturation*I + (1-saturation)*ones(3,1)*GSCL^T)   (MatExpr, float)
    const float g[3] = {0.0820f, 0.6094f, 0.3086f};
    float       A[3][3], B[3][3], M[3][3];
    float       oms = 1 - saturation;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            A[i][j] = i == j ? saturation : 0.f;
            B[i][j] = (float)((double)oms * (double)g[j]);
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            if (brightness == 1.0f) M[i][j] = A[i][j] + B[i][j];            // cv::add
            else M[i][j] = (float)((double)A[i][j] * brightness + (double)B[i][j] * brightness + 0.0);
        }                                                                    // cv::addWeighted
    bool diag = true;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            if (i != j && std::fabs((double)M[i][j]) > FLT_EPSILON) diag = false;
    const int n = m.w * m.h;
    if (diag) { // diagtransform_8u: saturate_cast<uchar>(m*src + 0) in float
        for (int y = 0; y < m.h; y++) {
            uint8_t* p = m.row(y);
            for (int x = 0; x < m.w; x++, p += 3) {
                uint8_t t0 = sat_u8f(M[0][0] * p[0] + 0.f);
                uint8_t t1 = sat_u8f(M[1][1] * p[1] + 0.f);
                uint8_t t2 = sat_u8f(M[2][2] * p[2] + 0.f);
                p[0] = t0, p[1] = t1, p[2] = t2;
            }
        }
        (void)n;
        return;
    }
    const float MAX_M = 32.f;
    bool        fixpt = true;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            if (!(std::fabs(M[i][j]) < MAX_M)) fixpt = false;
    if (fixpt) { // transform_8u, 10-bit fixed point (SSE2 path and its scalar tail agree)
        int q[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) q[i][j] = sat_s16(cv_roundf(M[i][j] * 1024));
        const int r = cv_roundf((0.f + 0.5f) * 1024);
        for (int y = 0; y < m.h; y++) {
            uint8_t* p = m.row(y);
            for (int x = 0; x < m.w; x++, p += 3) {
                int v0 = p[0], v1 = p[1], v2 = p[2];
                p[0] = sat_u8((q[0][0] * v0 + q[0][1] * v1 + q[0][2] * v2 + r) >> 10);
                p[1] = sat_u8((q[1][0] * v0 + q[1][1] * v1 + q[1][2] * v2 + r) >> 10);
                p[2] = sat_u8((q[2][0] * v0 + q[2][1] * v1 + q[2][2] * v2 + r) >> 10);
            }
        }
    } else { // transform_<uchar,float>
        for (int y = 0; y < m.h; y++) {
            uint8_t* p = m.row(y);
            for (int x = 0; x < m.w; x++, p += 3) {
                float v0 = p[0], v1 = p[1], v2 = p[2];
                uint8_t t0 = sat_u8f(M[0][0] * v0 + M[0][1] * v1 + M[0][2] * v2 + 0.f);
                uint8_t t1 = sat_u8f(M[1][0] * v0 + M[1][1] * v1 + M[1][2] * v2 + 0.f);
                uint8_t t2 = sat_u8f(M[2][0] * v0 + M[2][1] * v1 + M[2][2] * v2 + 0.f);
                p[0] = t0, p[1] = t1, p[2] = t2;
            }
        }
    }
}

// cvtColor BGR2HSV (RGB2HSV_b, hrange 180) -> hue shift -> HSV2BGR (HSV2RGB_b over HSV2RGB_f)
struct HsvTables {
    int sdiv[256], hdiv180[256];
    HsvTables()
    {
        sdiv[0] = hdiv180[0] = 0;
        for (int i = 1; i < 256; i++) {
            sdiv[i]    = cv_round((255 << 12) / (1. * i));
            hdiv180[i] = cv_round((180 << 12) / (6. * i));
        }
    }
};
const HsvTables& hsv_tables()
{
    static HsvTables t;
    return t;
}

void hue_shift_pixel(uint8_t* px, int hue)
{
    const HsvTables& T = hsv_tables();
    // RGB2HSV_b, bidx = 0 (BGR)
    int b = px[0], g = px[1], r = px[2];
    int v = std::max(b, std::max(g, r)), vmin = std::min(b, std::min(g, r));
    int diff = v - vmin;
    int vr = v == r ? -1 : 0, vg = v == g ? -1 : 0;
    int s = (diff * T.sdiv[v] + (1 << 11)) >> 12;
    int h = (vr & (g - b)) + (~vr & ((vg & (b - r + 2 * diff)) + ((~vg) & (r - g + 4 * diff))));
    h = (h * T.hdiv180[diff] + (1 << 11)) >> 12;
    h += h < 0 ? 180 : 0;
    uint8_t H = sat_u8(h), S = (uint8_t)s, V = (uint8_t)v;
    // image.cpp:386-390  *p = (*p + hue) % 180  (C remainder, stored as uchar)
    H = (uint8_t)((H + hue) % 180);
    // HSV2RGB_b: h stays 0..255, s and v scaled by 1/255; HSV2RGB_f with hscale = 6/180
    float hf = H, sf = S * (1.f / 255), vf = V * (1.f / 255);
    float bb, gg, rr;
    if (sf == 0) bb = gg = rr = vf;
    else {
        static const int sector_data[][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1},
                                             {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
        float tab[4];
        hf *= 6.f / 180.f;
        if (hf < 0) do hf += 6; while (hf < 0);
        else if (hf >= 6) do hf -= 6; while (hf >= 6);
        int sector = cv_floor(hf);
        hf -= sector;
        if ((unsigned)sector >= 6u) sector = 0, hf = 0.f;
        tab[0] = vf;
        tab[1] = vf * (1.f - sf);
        tab[2] = vf * (1.f - sf * hf);
        tab[3] = vf * (1.f - sf * (1.f - hf));
        bb = tab[sector_data[sector][0]];
        gg = tab[sector_data[sector][1]];
        rr = tab[sector_data[sector][2]];
    }
    px[0] = sat_u8f(bb * 255.f);
    px[1] = sat_u8f(gg * 255.f);
    px[2] = sat_u8f(rr * 255.f);
}

void cbsjitter(Img& m, float contrast, float brightness, float saturation, int hue)
{
    if (brightness != 1.0 || saturation != 1.0) bs_transform(m, brightness, saturation);
    if (hue != 0) {
        for (int y = 0; y < m.h; y++) {
            uint8_t* p = m.row(y);
            for (int x = 0; x < m.w; x++) hue_shift_pixel(p + 3 * x, hue);
        }
    }
    if (contrast != 1.0) {
        // cv::mean: exact per-channel sum times 1./N; dst = f32(x*c) (convertTo, f32 work type);
        // dst += (1.0-c)*mean runs with an f64 work type (same arithm_op rule that the
        // standardize goldens pin) and rounds to f32; convertTo(CV_8UC3) rounds half-even.
        long long sum[3] = {0, 0, 0};
        for (int y = 0; y < m.h; y++) {
            const uint8_t* p = m.row(y);
            for (int x = 0; x < m.w; x++)
                for (int k = 0; k < 3; k++) sum[k] += p[3 * x + k];
        }
        const double inv_n = 1. / (double)(m.w * m.h);
        double       shift[3];
        for (int k = 0; k < 3; k++) shift[k] = (1.0 - contrast) * ((double)sum[k] * inv_n);
        for (int y = 0; y < m.h; y++) {
            uint8_t* p = m.row(y);
            for (int x = 0; x < 3 * m.w; x++) {
                float t = (float)p[x] * contrast + 0.f;
                p[x]    = sat_u8f((float)((double)t + shift[x % 3]));
            }
        }
    }
}

// ---- photometric::lighting (src/image.cpp:320-346) ------------------------------------------
const float CPCA[3][3] = {{0.39731118f, 0.70119634f, -0.59200296f},
                          {-0.81698062f, -0.02354167f, -0.57618440f},
                          {0.41795513f, -0.71257945f, -0.56351045f}};
const float CSTD[3]    = {19.72083305f, 37.09388853f, 121.78006099f};

void lighting(Img& m, const float* al, int n, float sigma)
{
    if (n <= 0) return;
    float v[3], px[3];
    for (int k = 0; k < 3; k++) v[k] = CSTD[k] * al[k];                     // CSTD.mul(alphas)
    for (int i = 0; i < 3; i++) px[i] = CPCA[i][0] * v[0] + CPCA[i][1] * v[1] + CPCA[i][2] * v[2];
    // (inout + pixel) / (1 + sigma) -> convertTo(u8, a) then add(Scalar(pixel*a)) in CV_32S
    const double a  = 1. / (1.0 + (double)sigma);
    const float  af = (float)a;
    int          li[3];
    for (int k = 0; k < 3; k++) li[k] = cv_round((double)px[k] * a);
    for (int y = 0; y < m.h; y++) {
        uint8_t* p = m.row(y);
        for (int x = 0; x < 3 * m.w; x++) {
            int t = sat_u8f((float)p[x] * af + 0.f);
            p[x]  = sat_u8(t + li[x % 3]);
        }
    }
}

void flip_h(Img& m)
{
    for (int y = 0; y < m.h; y++) {
        uint8_t* p = m.row(y);
        for (int x = 0; x < m.w / 2; x++)
            for (int k = 0; k < m.cn; k++) std::swap(p[x * m.cn + k], p[(m.w - 1 - x) * m.cn + k]);
    }
}

// image::rotate (src/image.cpp:53-75): cv::getRotationMatrix2D(Point2i(cols/2, rows/2), angle,
// 1.0) and cv::warpAffine(..., input.size(), INTER_LINEAR | INTER_NEAREST, BORDER_CONSTANT, 0),
// restated from OpenCV 2.4 imgwarp.cpp:
//  * the forward matrix is inverted in double (warpAffine without WARP_INVERSE_MAP);
//  * per output pixel, with AB_BITS = 10, INTER_BITS = 5:
//      X = cvRound((M1*y + M2)*1024) + round_delta + cvRound(M0*x*1024)   (likewise Y)
//    round_delta = 512 (nearest) or 16 (linear); nearest takes (X >> 10, Y >> 10), linear takes
//    (X >> 5 >> 5, Y >> 5 >> 5) plus the 5-bit fractions (X & 31, Y & 31);
//  * remapBilinear: 15-bit weights from the 32x32 table initInterTab2D builds -- (32-fy)(32-fx)*32
//    etc.; the (0,0) entry saturates to 32767 and its correction lands on the fourth tap:
//    {32767, 0, 0, 1} -- then (sum + 2^14) >> 15; taps outside the image read the border 0.
void rotation_inverse_map(int w, int h, int angle, double M[6])
{
    const float  cx = (float)(w / 2), cy = (float)(h / 2); // Point2i -> Point2f
    const double a  = (double)angle * (3.1415926535897932384626433832795 / 180);
    const double alpha = std::cos(a) * 1.0, beta = std::sin(a) * 1.0;
    M[0] = alpha;
    M[1] = beta;
    M[2] = (1 - alpha) * cx - beta * cy;
    M[3] = -beta;
    M[4] = alpha;
    M[5] = beta * cx + (1 - alpha) * cy;
    double D = M[0] * M[4] - M[1] * M[3];
    D        = D != 0 ? 1. / D : 0;
    const double A11 = M[4] * D, A22 = M[0] * D;
    M[0] = A11;
    M[1] *= -D;
    M[3] *= -D;
    M[4] = A22;
    const double b1 = -M[0] * M[2] - M[1] * M[5];
    const double b2 = -M[3] * M[2] - M[4] * M[5];
    M[2] = b1;
    M[5] = b2;
}

static int sat_short(int v) { return std::min(std::max(v, -32768), 32767); }

Img rotate(const Img& in, int angle, bool interpolate)
{
    Img out = Img::alloc(in.w, in.h, in.cn);
    if (angle == 0) {
        for (int y = 0; y < in.h; y++) std::memcpy(out.row(y), in.row(y), (size_t)in.w * in.cn);
        return out;
    }
    double M[6];
    rotation_inverse_map(in.w, in.h, angle, M);
    const int        W = in.w, H = in.h, cn = in.cn;
    std::vector<int> ad(W), bd(W);
    for (int x = 0; x < W; x++) {
        ad[x] = cv_round(M[0] * x * 1024);
        bd[x] = cv_round(M[3] * x * 1024);
    }
    const int rdelta = interpolate ? 1024 / 32 / 2 : 1024 / 2;
    auto      tap    = [&](int xx, int yy, int c) -> int {
        return (xx >= 0 && xx < W && yy >= 0 && yy < H) ? in.row(yy)[xx * cn + c] : 0;
    };
    for (int y = 0; y < H; y++) {
        const int X0 = cv_round((M[1] * y + M[2]) * 1024) + rdelta;
        const int Y0 = cv_round((M[4] * y + M[5]) * 1024) + rdelta;
        uint8_t*  d  = out.row(y);
        for (int x = 0; x < W; x++) {
            if (!interpolate) {
                const int sx = sat_short((X0 + ad[x]) >> 10), sy = sat_short((Y0 + bd[x]) >> 10);
                for (int c = 0; c < cn; c++) d[x * cn + c] = (uint8_t)tap(sx, sy, c);
                continue;
            }
            const int X = (X0 + ad[x]) >> 5, Y = (Y0 + bd[x]) >> 5;
            const int sx = sat_short(X >> 5), sy = sat_short(Y >> 5);
            const int fx = X & 31, fy = Y & 31;
            int       w[4];
            if (fx == 0 && fy == 0) {
                w[0] = 32767, w[1] = 0, w[2] = 0, w[3] = 1;
            } else {
                w[0] = (32 - fy) * (32 - fx) * 32, w[1] = (32 - fy) * fx * 32;
                w[2] = fy * (32 - fx) * 32, w[3] = fy * fx * 32;
            }
            for (int c = 0; c < cn; c++) {
                const int v = tap(sx, sy, c) * w[0] + tap(sx + 1, sy, c) * w[1] + tap(sx, sy + 1, c) * w[2] +
                              tap(sx + 1, sy + 1, c) * w[3];
                d[x * cn + c] = (uint8_t)std::min(std::max((v + (1 << 14)) >> 15, 0), 255);
            }
        }
    }
    return out;
}

// image::transformer::transform_single_image (src/etl_image.cpp:146-202)
Img transform_single_image(const Img& src, const orc_params& p)
{
    Img rot;
    Img base = Img::view(src.data, src.w, src.h, src.cn, src.stride);
    if (p.angle != 0) { // image::rotate, interpolated (etl_image.cpp:150-151)
        rot  = rotate(base, p.angle, true);
        base = Img::view(rot.data, rot.w, rot.h, rot.cn, rot.stride);
    }
    Img ex;
    if (p.expand_ratio > 1.0f) { // image::expand (image.cpp:276-303), etl_image.cpp:155-159
        if (p.expand_x < 0 || p.expand_y < 0 || base.w + p.expand_x > p.expand_w || base.h + p.expand_y > p.expand_h)
            throw std::invalid_argument("Invalid parameters to expand image");
        ex = Img::alloc(p.expand_w, p.expand_h, base.cn);
        for (int y = 0; y < base.h; y++)
            std::memcpy(ex.row(y + p.expand_y) + (size_t)p.expand_x * base.cn, base.row(y), (size_t)base.w * base.cn);
        base = Img::view(ex.data, ex.w, ex.h, ex.cn, ex.stride);
    }
    Img rs;
    if (p.resize_short_size != 0) {
        int rw, rh;
        resized_short_size(base.w, base.h, p.resize_short_size, &rw, &rh);
        rs = Img::alloc(rw, rh, src.cn);
        resize_cv(base, rs, p.interp); // image::resize_short: cv::resize, no same-size shortcut
        base = Img::view(rs.data, rs.w, rs.h, rs.cn, rs.stride);
    }
    if (p.crop_x < 0 || p.crop_y < 0 || p.crop_w <= 0 || p.crop_h <= 0 ||
        p.crop_x + p.crop_w > base.w || p.crop_y + p.crop_h > base.h)
        throw std::invalid_argument("cropbox outside image");
    Img crop = Img::view(base.row(p.crop_y) + (size_t)p.crop_x * base.cn, p.crop_w, p.crop_h,
                         base.cn, base.stride);
    Img padded;
    if (!(p.padding == 0 || (p.pad_off_x == p.padding && p.pad_off_y == p.padding))) {
        // image::add_padding (image.cpp:77-91): zero border, then crop back to the input size
        padded = Img::alloc(crop.w, crop.h, crop.cn);
        for (int y = 0; y < crop.h; y++)
            for (int x = 0; x < crop.w; x++) {
                int sx = x + p.pad_off_x - p.padding, sy = y + p.pad_off_y - p.padding;
                if (sx < 0 || sy < 0 || sx >= crop.w || sy >= crop.h) continue;
                std::memcpy(padded.row(y) + x * crop.cn, crop.row(sy) + sx * crop.cn, crop.cn);
            }
        crop = Img::view(padded.data, padded.w, padded.h, padded.cn, padded.stride);
    }
    Img out = Img::alloc(p.out_w, p.out_h, src.cn);
    resize_any(crop, out, p.interp);
    if (src.cn == 3) {
        cbsjitter(out, p.contrast, p.brightness, p.saturation, p.hue);
        lighting(out, p.lighting, p.n_lighting, p.color_noise_std);
    }
    if (p.flip) flip_h(out);
    return out;
}

// image::standardize arithmetic (image.cpp:129-174 + OpenCV 2.4 arithm_op): every
// Mat(f32) op Scalar(f64) runs with an f64 work type and rounds back to f32 after each op.
// Pinned bit-exact by augment_output_linear_{train,eval}.bin (all 765 channel/value pairs).
float standardize_value(int x, double mean, double stddev)
{
    float t1 = (float)((double)(float)x * (1. / 255.));
    float t2 = (float)((double)t1 - mean);
    if (stddev == 0) return t2;
    return (float)((double)t2 * (1. / stddev));
}

// image::loader::load (src/etl_image.cpp:246-341), non-fixed-aspect-ratio branch
void load_image(const Img& img, const orc_load_config& lc, void* out)
{
    const int cn = lc.channels, w = img.w, h = img.h;
    if (img.cn != cn) throw std::invalid_argument("channel mismatch");
    const size_t plane = (size_t)w * h;
    for (int y = 0; y < h; y++) {
        const uint8_t* p = img.row(y);
        for (int x = 0; x < w; x++) {
            for (int oc = 0; oc < cn; oc++) {
                int    sc  = lc.bgr_to_rgb ? (cn - 1 - oc) : oc; // from_to {0,2,1,1,2,0}
                int    v   = p[x * cn + sc];
                size_t idx = lc.channel_major ? (size_t)oc * plane + (size_t)y * w + x
                                              : ((size_t)y * w + x) * cn + oc;
                // convert_mix_channels (image.cpp:176-212): Mat::convertTo(target type) of the
                // uint8 record, saturating, then standardize (float / double only, image.cpp:129-174)
                switch (lc.out_dtype) {
                case 0: ((uint8_t*)out)[idx] = (uint8_t)v; break;              // CV_8U
                case 2: ((int8_t*)out)[idx] = (int8_t)std::min(v, 127); break;  // CV_8S (int8_t, char)
                case 3: ((int16_t*)out)[idx] = (int16_t)v; break;              // CV_16S
                case 4: ((uint16_t*)out)[idx] = (uint16_t)v; break;            // CV_16U
                case 5: ((int32_t*)out)[idx] = v; break;                       // CV_32S (int32_t, uint32_t)
                case 6: { // CV_64F: multiply / subtract / multiply in double, nothing rounded to float
                    double d = (double)v;
                    if (lc.has_mean) {
                        d = d * (1. / 255.) - lc.mean[oc];
                        if (lc.stddev[oc] != 0) d = d * (1. / lc.stddev[oc]);
                    }
                    ((double*)out)[idx] = d;
                    break;
                }
                default: { // CV_32F
                    float f = lc.has_mean ? standardize_value(v, lc.mean[oc], lc.stddev[oc]) : (float)v;
                    ((float*)out)[idx] = f;
                }
                }
            }
        }
    }
}

// pixel_mask::transformer::transform (src/etl_pixel_mask.cpp:65-92)
Img transform_mask(const Img& src, const orc_params& p)
{
    Img rot;
    Img base = Img::view(src.data, src.w, src.h, src.cn, src.stride);
    if (p.angle != 0) { // image::rotate(..., interpolate=false, border 0) (etl_pixel_mask.cpp:72-74)
        rot  = rotate(base, p.angle, false);
        base = Img::view(rot.data, rot.w, rot.h, rot.cn, rot.stride);
    }
    if (p.crop_x < 0 || p.crop_y < 0 || p.crop_w <= 0 || p.crop_h <= 0 ||
        p.crop_x + p.crop_w > base.w || p.crop_y + p.crop_h > base.h)
        throw std::invalid_argument("cropbox outside mask");
    Img crop = Img::view(base.row(p.crop_y) + (size_t)p.crop_x * base.cn, p.crop_w, p.crop_h,
                         base.cn, base.stride);
    Img out = Img::alloc(p.out_w, p.out_h, src.cn);
    resize_any(crop, out, 1);
    if (p.flip) flip_h(out);
    return out;
}

template <typename F>
int guarded(F&& f)
{
    try {
        f();
        return 0;
    } catch (const std::exception& e) {
        g_err = e.what();
        return -1;
    }
}

} // namespace

// transpose_regular<T> (src/buffer_batch.cpp:186-200): walks the destination in order, reading
// the source down each column.  (transpose_buf's SSE variant for 16-aligned sizes computes the
// same permutation.)
template <typename T>
static void transpose_regular(T* dest, const T* src, int64_t rows, int64_t cols)
{
    int64_t dst_indx = 0;
    for (int64_t c = 0; c < cols; ++c) {
        int64_t src_indx = c;
        for (int64_t r = 0; r < rows; ++r) {
            dest[dst_indx++] = src[src_indx];
            src_indx += cols;
        }
    }
}

extern "C" {

void* orc_factory_create(const orc_aug_config* cfg) { return new Factory(*cfg); }
void  orc_factory_destroy(void* f) { delete (Factory*)f; }

// sampler::sample_patch + batch_sampler::sample_patches (src/augment_image.cpp:359-395, 567-586)
void sample_patches(const orc_batch_sampler& bs, Engine& e, const std::vector<NBox>& objs, std::vector<NBox>& samples)
{
    std::uniform_real_distribution<float> sd{bs.scale_min, bs.scale_max};
    int found = 0;
    for (unsigned t = 0; t < (unsigned)bs.max_trials; t++) {
        if (bs.max_sample != -1 && found >= bs.max_sample) break;
        float s   = sd(e);
        float amn = std::max<float>(bs.ar_min, std::pow(s, 2.));
        float amx = std::min<float>(bs.ar_max, 1 / std::pow(s, 2.));
        float ar  = std::uniform_real_distribution<float>(amn, amx)(e);
        float bw = s * std::sqrt(ar), bh = s / std::sqrt(ar);
        float wo = std::uniform_real_distribution<float>(0.f, 1.f - bw)(e);
        float ho = std::uniform_real_distribution<float>(0.f, 1.f - bh)(e);
        NBox  nb = make_nbox(wo, ho, wo + bw, ho + bh);
        if (satisfies(bs, nb, objs)) found++, samples.push_back(nb);
    }
}

int orc_sample_patches(void* fp, int sampler, uint32_t* state, const float* nboxes, int n, float* out, int cap,
                       int* n_out)
{
    return guarded([&] {
        Factory& f = *(Factory*)fp;
        if (sampler < 0 || sampler >= f.c.n_samplers) throw std::invalid_argument("sampler index");
        Engine            e(*state);
        std::vector<NBox> objs, samples;
        for (int i = 0; i < n; i++) objs.push_back(make_nbox(nboxes[4 * i], nboxes[4 * i + 1], nboxes[4 * i + 2], nboxes[4 * i + 3]));
        sample_patches(f.c.samplers[sampler], e, objs, samples);
        *n_out = (int)samples.size();
        for (int i = 0; i < (int)samples.size() && i < cap; i++) {
            out[4 * i] = samples[i].x0, out[4 * i + 1] = samples[i].y0;
            out[4 * i + 2] = samples[i].x1, out[4 * i + 3] = samples[i].y1;
        }
        *state = e.last;
    });
}

int orc_make_ssd_params(void* fp, uint32_t* state, int in_w, int in_h, int out_w, int out_h, const float* boxes,
                        int n_boxes, orc_params* out)
{
    return guarded([&] {
        Factory& f = *(Factory*)fp;
        Engine   e(*state);
        make_params(f, e, in_w, in_h, out_w, out_h, out);
        out->out_w = out_w, out->out_h = out_h;
        std::uniform_real_distribution<float> ratio_d{f.c.expand_ratio_min, f.c.expand_ratio_max}, unit{0.0f, 1.0f};
        float      ratio   = ratio_d(e);
        const bool enabled = unit(e) < f.c.expand_probability;
        if (ratio < 1.) throw std::invalid_argument("Expand ratio must be greater than 1.");
        int ox = 0, oy = 0, ew = in_w, eh = in_h;
        if (enabled) {
            float fw = ratio * (float)in_w, fh = ratio * (float)in_h;
            ew = (int)std::floor(fw), eh = (int)std::floor(fh);
            float wo = unit(e) * (fw - (float)in_w);
            float ho = unit(e) * (fh - (float)in_h);
            ox = (int)std::floor(wo), oy = (int)std::floor(ho);
        } else {
            ratio = 1.0f;
        }
        out->expand_ratio = ratio, out->expand_x = ox, out->expand_y = oy, out->expand_w = ew, out->expand_h = eh;
        std::vector<NBox> objs;
        for (int i = 0; i < n_boxes; i++) {
            const float* b = boxes + 4 * i;
            if (b[2] + ox > ew || b[3] + oy > eh) throw std::invalid_argument("Invalid parameters to expand boundingbox");
            objs.push_back(make_nbox((b[0] + ox) / ew, (b[1] + oy) / eh, (b[2] + ox + 1) / ew, (b[3] + oy + 1) / eh));
        }
        if (!f.c.crop_enable) {
            std::vector<NBox> samples;
            for (int k = 0; k < f.c.n_samplers; k++) sample_patches(f.c.samplers[k], e, objs, samples);
            NBox patch{0, 0, 1, 1};
            if (!samples.empty()) patch = samples[std::uniform_int_distribution<int>(0, (int)samples.size() - 1)(e)];
            float x0 = patch.x0 * (float)ew, y0 = patch.y0 * (float)eh;
            float x1 = patch.x1 * (float)ew - 1, y1 = patch.y1 * (float)eh - 1;
            out->crop_x = (int)std::round(x0), out->crop_y = (int)std::round(y0);
            out->crop_w = (int)std::round(x1 - x0 + 1), out->crop_h = (int)std::round(y1 - y0 + 1);
        }
        *state = e.last;
    });
}

int orc_make_params(void* f, uint32_t* state, int in_w, int in_h, int out_w, int out_h,
                    orc_params* out)
{
    return guarded([&] {
        Engine e(*state);
        make_params(*(Factory*)f, e, in_w, in_h, out_w, out_h, out);
        *state = e.last;
    });
}

int   orc_unbiased_round(float x) { return unbiased_round(x); }
float orc_calculate_scale(int w, int h, int ow, int oh) { return calculate_scale(w, h, ow, oh); }
void  orc_cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* rw, float* rh)
{
    cropbox_max_proportional(in_w, in_h, out_w, out_h, rw, rh);
}

void orc_seed_slots(uint32_t seed, int n, uint32_t* states)
{
    // engine_i.seed(generator_seed()): minstd's seed(s) keeps s mod m (1 if that is 0),
    // so the state word of slot i is the i-th output of minstd_rand0(seed).
    std::minstd_rand0 g(seed);
    for (int i = 0; i < n; i++) {
        uint32_t s = g() % 2147483647u;
        states[i]  = s == 0 ? 1 : s;
    }
}

int orc_transform_image(const uint8_t* src, int w, int h, int cn, int stride, const orc_params* p,
                        uint8_t* out)
{
    return guarded([&] {
        Img s = Img::view(src, w, h, cn, stride);
        Img o = transform_single_image(s, *p);
        std::memcpy(out, o.data, (size_t)o.w * o.h * o.cn);
    });
}

int orc_load_image(const uint8_t* img, int w, int h, const orc_load_config* lc, void* out)
{
    return guarded([&] { load_image(Img::view(img, w, h, lc->channels, w * lc->channels), *lc, out); });
}

int orc_transform_mask(const uint8_t* src, int w, int h, int stride, const orc_params* p,
                       uint8_t* out)
{
    return guarded([&] {
        Img o = transform_mask(Img::view(src, w, h, 1, stride), *p);
        std::memcpy(out, o.data, (size_t)o.w * o.h);
    });
}

int orc_resize_linear(const uint8_t* src, int sw, int sh, int sstride, int cn, uint8_t* dst, int dw,
                      int dh)
{
    return guarded([&] {
        Img s = Img::view(src, sw, sh, cn, sstride);
        Img d = Img::view(dst, dw, dh, cn, dw * cn);
        resize_linear(s, d);
    });
}

int orc_resize_nearest(const uint8_t* src, int sw, int sh, int sstride, int cn, uint8_t* dst,
                       int dw, int dh)
{
    return guarded([&] {
        Img s = Img::view(src, sw, sh, cn, sstride);
        Img d = Img::view(dst, dw, dh, cn, dw * cn);
        resize_nearest(s, d);
    });
}

// cv::resize with any of aeon's interpolation methods (0 LINEAR, 1 NEAREST, 2 CUBIC, 3 AREA, 4 LANCZOS4)
int orc_resize_cv(const uint8_t* src, int sw, int sh, int sstride, int cn, uint8_t* dst, int dw, int dh, int interp)
{
    return guarded([&] {
        if (interp < 0 || interp > 4) throw std::invalid_argument("unknown interpolation");
        Img s = Img::view(src, sw, sh, cn, sstride);
        Img d = Img::view(dst, dw, dh, cn, dw * cn);
        resize_cv(s, d, interp);
    });
}

// interpolateLanczos4's coefficients of fraction x (the product builds them on the host too)
void orc_lanczos4_coeffs(float x, float* out) { interpolate_lanczos4(x, out); }

void orc_cbsjitter(uint8_t* img, int w, int h, float contrast, float brightness, float saturation,
                   int hue)
{
    Img m = Img::view(img, w, h, 3, w * 3);
    cbsjitter(m, contrast, brightness, saturation, hue);
}

void orc_lighting(uint8_t* img, int w, int h, const float* l, int n, float sigma)
{
    Img m = Img::view(img, w, h, 3, w * 3);
    lighting(m, l, n, sigma);
}

// image::standardize applied to a CV_8U canvas (the fixed_aspect_ratio loader standardizes its
// uint8 planes in place, etl_image.cpp:263-300): OpenCV 2.4 arithm_op on 8U data --
// multiply(x, 1/255.) in double then saturate_cast<uchar>; subtract(scalar mean) with the scalar
// converted to int first (cvRound: "just one input is floating-point" rule for add/sub);
// multiply(1/stddev) in double, saturating.  Parity unpinned: no reference fixture covers it.
int orc_u8_standardize_value(int x, double mean, double stddev)
{
    int a = sat_u8(cv_round((double)x * (1. / 255.)));
    a     = sat_u8(a - cv_round(mean));
    if (stddev != 0) a = sat_u8(cv_round((double)a * (1. / stddev)));
    return a;
}

float orc_standardize_value(int x, double mean, double stddev)
{
    return standardize_value(x, mean, stddev);
}

// CPU baseline: aeon's thread_pool policy -- N workers pulling record indices from one
// atomic counter (src/thread_pool.hpp:155-162), each running transform + load per record.
int orc_rotate(const uint8_t* src, int w, int h, int cn, int stride, int angle, int interpolate, uint8_t* out)
{
    return guarded([&] {
        Img o = rotate(Img::view(src, w, h, cn, stride), angle, interpolate != 0);
        std::memcpy(out, o.data, (size_t)w * h * cn);
    });
}

} // extern "C"

namespace {
// The CPU baseline's pool: aeon's thread_pool (src/thread_pool.hpp:133-138) pins worker t to
// thread_affinity_map[t]; orc_set_affinity installs that map (worker t -> cpus[t % n]), none = unpinned.
std::vector<int> g_affinity;

template <typename W>
void run_pool(int threads, W&& work)
{
    std::vector<std::thread> pool;
    for (int t = 0; t < std::max(1, threads); t++)
        pool.emplace_back([&, t] {
            if (!g_affinity.empty()) {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(g_affinity[t % g_affinity.size()], &set);
                (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
            }
            work(t);
        });
    for (auto& t : pool) t.join();
}
} // namespace

extern "C" {

void orc_set_affinity(const int* cpus, int n)
{
    g_affinity.assign(cpus, cpus + std::max(0, n));
}

// worker t of a `threads` pool: the CPU its sched_getaffinity holds when that is exactly one, else -1
void orc_pool_cpus(int threads, int* out)
{
    run_pool(threads, [&](int t) {
        cpu_set_t set;
        out[t] = -1;
        if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) == 1)
            for (int c = 0; c < CPU_SETSIZE; c++)
                if (CPU_ISSET(c, &set)) out[t] = c;
    });
}

double orc_batch_augment(int n, const uint8_t* const* srcs, const int* widths, const int* heights,
                         const orc_params* params, const orc_load_config* lc, void* out,
                         size_t item_bytes, int threads)
{
    std::atomic<int>  next{0};
    std::atomic<bool> failed{false};
    auto              work = [&] {
        for (;;) {
            int i = next.fetch_add(1);
            if (i >= n) break;
            try {
                Img s = Img::view(srcs[i], widths[i], heights[i], lc->channels,
                                  widths[i] * lc->channels);
                Img o = transform_single_image(s, params[i]);
                load_image(o, *lc, (char*)out + (size_t)i * item_bytes);
            } catch (const std::exception& e) {
                g_err = e.what();
                failed = true;
            }
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    run_pool(threads, [&](int) { work(); });
    auto t1 = std::chrono::steady_clock::now();
    if (failed) return -1.0;
    return std::chrono::duration<double>(t1 - t0).count();
}

double orc_batch_image_mask(int n, const uint8_t* const* srcs, const uint8_t* const* masks, const int* widths,
                            const int* heights, const orc_params* params, const orc_load_config* lc,
                            void* out, size_t item_bytes, const orc_load_config* mlc, void* mout,
                            size_t mitem_bytes, int threads)
{
    std::atomic<int>  next{0};
    std::atomic<bool> failed{false};
    auto              work = [&] {
        for (;;) {
            int i = next.fetch_add(1);
            if (i >= n) break;
            try {
                Img s = Img::view(srcs[i], widths[i], heights[i], lc->channels, widths[i] * lc->channels);
                load_image(transform_single_image(s, params[i]), *lc, (char*)out + (size_t)i * item_bytes);
                Img m = Img::view(masks[i], widths[i], heights[i], 1, widths[i]);
                load_image(transform_mask(m, params[i]), *mlc, (char*)mout + (size_t)i * mitem_bytes);
            } catch (const std::exception& e) {
                g_err  = e.what();
                failed = true;
            }
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    run_pool(threads, [&](int) { work(); });
    auto t1 = std::chrono::steady_clock::now();
    if (failed) return -1.0;
    return std::chrono::duration<double>(t1 - t0).count();
}

// aeon's whole CPU path per record -- image::extractor::extract (JPEG decode, jpeg_oracle.cpp) ->
// transform_single_image -> loader::load -- over a batch of encoded files on a thread pool: the CPU
// baseline of the end-to-end decode stage.  params[i] must be drawn for file i's decoded size.
double orc_batch_decode_augment(int n, const uint8_t* const* files, const size_t* sizes, const orc_params* params,
                                const orc_load_config* lc, void* out, size_t item_bytes, int threads)
{
    std::atomic<int>  next{0};
    std::atomic<bool> failed{false};
    auto              work = [&] {
        std::vector<uint8_t> px;
        for (;;) {
            int i = next.fetch_add(1);
            if (i >= n) break;
            int w, h, nc;
            if (orc_jpeg_info(files[i], sizes[i], &w, &h, &nc) != 0) {
                g_err  = orc_jpeg_last_error();
                failed = true;
                continue;
            }
            px.resize((size_t)w * h * lc->channels);
            if (orc_jpeg_decode(files[i], sizes[i], lc->channels, px.data()) != 0) {
                g_err  = orc_jpeg_last_error();
                failed = true;
                continue;
            }
            try {
                Img o = transform_single_image(Img::view(px.data(), w, h, lc->channels, w * lc->channels), params[i]);
                load_image(o, *lc, (char*)out + (size_t)i * item_bytes);
            } catch (const std::exception& e) {
                g_err  = e.what();
                failed = true;
            }
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    run_pool(threads, [&](int) { work(); });
    auto t1 = std::chrono::steady_clock::now();
    if (failed) return -1.0;
    return std::chrono::duration<double>(t1 - t0).count();
}

int orc_transpose(void* dest, const void* src, int64_t rows, int64_t cols, int element_size)
{
    switch (element_size) {
    case 1: transpose_regular((uint8_t*)dest, (const uint8_t*)src, rows, cols); return 0;
    case 2: transpose_regular((uint16_t*)dest, (const uint16_t*)src, rows, cols); return 0;
    case 4: transpose_regular((uint32_t*)dest, (const uint32_t*)src, rows, cols); return 0;
    case 8: transpose_regular((uint64_t*)dest, (const uint64_t*)src, rows, cols); return 0;
    default: g_err = "unsupported datatype for transpose"; return -1;
    }
}

const char* orc_last_error(void) { return g_err.c_str(); }

} // extern "C"
