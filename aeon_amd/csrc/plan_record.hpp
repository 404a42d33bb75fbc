// plan_record.hpp -- the per-record arithmetic aeon does on the host before touching pixels
// (cv::resize dispatch, cropbox window, cv::transform matrix, lighting pixel): the host planner's
// (stage.cpp) job of one record, built with -ffp-contract=off so every float/double expression
// rounds as aeon's x86 build does.
#pragma once
#include <stdint.h>

#include <cfloat>

#include "../../include/aeon_hip.h"
#include "aug_job.hpp"

namespace aeon_hip {

AEON_HD inline int rint_d(double v) { return (int)__builtin_rint(v); } // cvRound (round half to even)
AEON_HD inline int rint_f(float v) { return (int)__builtin_rintf(v); }

// OpenCV 2.4 cv::resize dispatch for 8U: INTER_NEAREST, 2x INTER_LINEAR -> INTER_AREA's fast path,
// generic INTER_LINEAR.  An identity resize (image::resize's same-size shortcut) is planned as
// LINEAR / NEAREST: with scale 1 every LINEAR tap is (sx = dx, weights 2048/0), which reproduces
// the source exactly through both OpenCV vertical formulas, so no separate copy launch is needed.
AEON_HD inline int choose_mode(int sw, int sh, int dw, int dh, int interp, int cn)
{
    if (interp == AEON_INTERP_NEAREST) return RESIZE_NEAREST;
    if (sw == dw && sh == dh) return RESIZE_LINEAR;
    const double sx = 1. / ((double)dw / sw), sy = 1. / ((double)dh / sh);
    const int    ix = rint_d(sx), iy = rint_d(sy);
    const bool   fast = __builtin_fabs(sx - ix) < DBL_EPSILON && __builtin_fabs(sy - iy) < DBL_EPSILON;
    if (fast && ix == 2 && iy == 2 && (cn == 1 || cn == 3)) return RESIZE_AREA2X;
    return RESIZE_LINEAR;
}

// First element of a W-element destination row handled by OpenCV's scalar tail after
// VResizeLinearVec_32s8u (16-wide loop while x <= W-16, 4-wide while x < W-4).
AEON_HD inline int simd_boundary(int W)
{
    int x = W >= 16 ? (W / 16) * 16 : 0;
    while (x < W - 4) x += 4;
    return x;
}

// photometric::cbsjitter brightness/saturation matrix (src/image.cpp:362-373) and the
// cv::transform path OpenCV 2.4 picks for it.
AEON_HD inline void plan_bs(AugJob& J, float brightness, float saturation)
{
    const float g[3] = {0.0820f, 0.6094f, 0.3086f};
    float       M[9];
    const float oms = 1 - saturation;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const float A = i == j ? saturation : 0.f;
            const float B = (float)((double)oms * (double)g[j]);
            M[i * 3 + j] = brightness == 1.0f ? A + B : (float)((double)A * brightness + (double)B * brightness + 0.0);
        }
    bool diag = true;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            if (i != j && __builtin_fabs((double)M[i * 3 + j]) > FLT_EPSILON) diag = false;
    bool fixpt = true;
    for (int k = 0; k < 9; k++)
        if (!(__builtin_fabsf(M[k]) < 32.f)) fixpt = false;
    for (int k = 0; k < 9; k++) {
        J.bsm[k]   = M[k];
        const int q = rint_f(M[k] * 1024);
        J.bsq[k]   = q < -32768 ? -32768 : (q > 32767 ? 32767 : q);
    }
    J.bs_kind = diag ? BS_DIAG : (fixpt ? BS_FIXPT : BS_FLOAT);
}

// photometric::lighting (src/image.cpp:320-346): the PCA pixel and its (1+sigma) scaling.
AEON_HD inline void plan_lighting(AugJob& J, const float* al, float sigma)
{
    const float CPCA[3][3] = {{0.39731118f, 0.70119634f, -0.59200296f},
                              {-0.81698062f, -0.02354167f, -0.57618440f},
                              {0.41795513f, -0.71257945f, -0.56351045f}};
    const float CSTD[3]    = {19.72083305f, 37.09388853f, 121.78006099f};
    float       v[3], px[3];
    for (int k = 0; k < 3; k++) v[k] = CSTD[k] * al[k];
    for (int i = 0; i < 3; i++) px[i] = CPCA[i][0] * v[0] + CPCA[i][1] * v[1] + CPCA[i][2] * v[2];
    const double a = 1. / (1.0 + (double)sigma);
    J.light_a      = (float)a;
    for (int k = 0; k < 3; k++) J.light_add[k] = rint_d((double)px[k] * a);
}

// Photometric stages a record's params switch on (cbsjitter + lighting, src/image.cpp:336-406).
AEON_HD inline int photo_flags(const aeon_aug_params& p)
{
    int photo = 0;
    if (p.brightness != 1.0f || p.saturation != 1.0f) photo |= PHOTO_BS;
    if (p.hue != 0) photo |= PHOTO_HUE;
    if (p.contrast != 1.0f) photo |= PHOTO_CONTRAST;
    if (p.n_lighting > 0) photo |= PHOTO_LIGHTING;
    return photo;
}

// Loader geometry of the output buffer (image::loader, src/etl_image.cpp:246-341).
struct OutGeom {
    int32_t fixed_aspect_ratio, canvas_w, canvas_h;
};

// The record goes through image::expand (etl_image.cpp:155-159: expand_ratio > 1), a pre-pass.
AEON_HD inline bool expands(const aeon_aug_params& p) { return p.expand_ratio > 1.0f; }

// transform_single_image (src/etl_image.cpp:146-202) of one record read straight from its
// decoded source: crop [+ add_padding] -> resize -> [cbsjitter -> lighting] -> flip -> load, as ONE
// job.  Callers handle rotation / resize_short (pre-passes) and contrast (two passes) by patching
// the job this returns.  `out_item` is the record's output item; is_mask = pixel-mask transform
// (NEAREST, no padding, no photometric).  Inputs are assumed validated (stage.cpp).
AEON_HD inline void plan_direct(const aeon_img_desc& d, uint64_t src_base, const aeon_aug_params& p,
                                const OutGeom& o, uint64_t out_item, bool is_mask, AugJob& J)
{
    J            = AugJob{};
    const int cn = d.channels;
    J.src_ptr    = src_base + d.offset;
    J.src_bytes  = (uint64_t)d.stride * d.height;
    J.src_w = d.width, J.src_h = d.height, J.src_stride = d.stride, J.cn = cn;
    J.stats_slot = -1;
    J.crop_x = p.crop_x, J.crop_y = p.crop_y, J.crop_w = p.crop_w, J.crop_h = p.crop_h;
    if (!is_mask && !(p.padding == 0 || (p.pad_off_x == p.padding && p.pad_off_y == p.padding))) {
        J.shift_x = p.pad_off_x - p.padding;
        J.shift_y = p.pad_off_y - p.padding;
        J.padded  = 1;
    }
    J.mode    = choose_mode(J.crop_w, J.crop_h, p.out_w, p.out_h, is_mask ? AEON_INTERP_NEAREST : p.interp, cn);
    J.scale_x = 1. / ((double)p.out_w / J.crop_w);
    J.scale_y = 1. / ((double)p.out_h / J.crop_h);
    J.dst_w = p.out_w, J.dst_h = p.out_h;
    J.win_x = 0, J.win_y = 0, J.win_w = p.out_w, J.win_h = p.out_h;
    J.xv      = simd_boundary(p.out_w * cn);
    J.flip    = p.flip ? 1 : 0;
    J.out_ptr = out_item;
    // image::loader::load (etl_image.cpp:258-306): planes of the record's own size, or with
    // fixed_aspect_ratio the record at the top-left of the (zeroed) config-sized canvas
    J.out_pitch = o.fixed_aspect_ratio ? o.canvas_w : p.out_w;
    J.out_plane = o.fixed_aspect_ratio ? o.canvas_w * o.canvas_h : p.out_w * p.out_h;
    if (!is_mask) {
        const int photo = photo_flags(p);
        if (photo & PHOTO_BS) plan_bs(J, p.brightness, p.saturation);
        J.contrast = p.contrast;
        J.hue      = p.hue;
        if (photo & PHOTO_LIGHTING) plan_lighting(J, p.lighting, p.color_noise_std);
        J.photo = photo;
    }
}

} // namespace aeon_hip
