// param_factory.hpp -- augment::image::param_factory for the HIP stage (host C++).
//
// Same configuration keys, validators, distributions and RNG draw order as aeon's
// src/augment_image.hpp:125-249 / src/augment_image.cpp:28-230, so a record drawn from the
// same minstd_rand0 state gets the same params as in aeon.  Parameter sampling stays on the
// host (µs per record); the pixel work it parameterises runs on the GPU.
#pragma once
#include <random>
#include <string>
#include <vector>

#include "../../include/aeon_hip.h"
#include "json.hpp"

namespace aeon_hip {

class param_factory {
public:
    explicit param_factory(const Json& js);

    // src/augment_image.cpp:107-230
    template <typename URNG>
    void make_params(URNG& random, int in_w, int in_h, int out_w, int out_h, aeon_aug_params* p) const;

    bool                do_area_scale        = false;
    bool                crop_enable          = true;
    bool                fixed_aspect_ratio   = false;
    std::vector<double> mean;
    std::vector<double> stddev;
    int                 resize_short_size    = 0;
    std::string         interpolation_method = "LINEAR";
    float               expand_probability   = 0.f;
    float               fixed_scaling_factor = -1;
    int                 padding              = 0;
    std::string         debug_output_directory;
    bool                flip_enable = false;
    bool                center      = true;

    mutable std::uniform_real_distribution<float> scale{1.0f, 1.0f};
    mutable std::uniform_int_distribution<int>    angle{0, 0};
    mutable std::normal_distribution<float>       lighting{0.0f, 0.0f};
    mutable std::uniform_real_distribution<float> horizontal_distortion{1.0f, 1.0f};
    mutable std::uniform_real_distribution<float> contrast{1.0f, 1.0f};
    mutable std::uniform_real_distribution<float> brightness{1.0f, 1.0f};
    mutable std::uniform_real_distribution<float> saturation{1.0f, 1.0f};
    mutable std::uniform_real_distribution<float> expand_ratio{1.0f, 1.0f};
    mutable std::uniform_int_distribution<int>    hue{0, 0};
    mutable std::uniform_real_distribution<float> crop_offset{0.5f, 0.5f};
    mutable std::bernoulli_distribution           flip_distribution{0};
    mutable std::uniform_int_distribution<int>    padding_crop_offset_distribution{0, 0};

    int interp_code() const; // AEON_INTERP_* (or -1 for CUBIC/AREA/LANCZOS4)
};

// ---- geometry helpers (src/image.cpp:108-273, src/util.cpp:212-239) ---------------------------
int   unbiased_round(float x);
void  get_resized_short_size(int in_w, int in_h, int target, int* ow, int* oh);
float calculate_scale(int w, int h, int ow, int oh);
void  cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* rw, float* rh);
inline int cv_round(double v) { return (int)std::nearbyint(v); }
inline int cv_roundf(float v) { return (int)std::nearbyintf(v); }

template <typename URNG>
void param_factory::make_params(URNG& random, int in_w, int in_h, int out_w, int out_h,
                                aeon_aug_params* p) const
{
    *p            = aeon_aug_params{};
    p->out_w      = out_w;
    p->out_h      = out_h;
    p->angle      = angle(random);
    p->flip       = flip_distribution(random) ? 1 : 0;
    p->hue        = hue(random);
    p->contrast   = contrast(random);
    p->brightness = brightness(random);
    p->saturation = saturation(random);
    p->padding    = padding;
    p->resize_short_size = resize_short_size;
    p->interp            = interp_code();

    float isw = (float)in_w, ish = (float)in_h; // cv::Size2f input_size
    if (!crop_enable) {
        p->pad_off_x = padding_crop_offset_distribution(random);
        p->pad_off_y = padding_crop_offset_distribution(random);
        p->crop_x = 0, p->crop_y = 0;
        p->crop_w = cv_roundf(isw), p->crop_h = cv_roundf(ish);
        float s = fixed_scaling_factor > 0 ? fixed_scaling_factor
                                           : calculate_scale(in_w, in_h, out_w, out_h);
        isw *= s;
        ish *= s;
        p->out_w = unbiased_round(isw);
        p->out_h = unbiased_round(ish);
    } else if (do_area_scale) {
        float hd = horizontal_distortion(random);
        hd       = std::sqrt(hd);
        float sw = hd, sh = 1 / hd;
        float bound = std::min((float)in_w / (float)in_h / (sw * sw),
                               (float)in_h / (float)in_w / (sh * sh));
        float smax = std::min(scale.max(), bound);
        float smin = std::min(scale.min(), bound);
        std::uniform_real_distribution<float> scale2{smin, smax};
        float ta = std::sqrt((float)((size_t)in_h * (size_t)in_w) * scale2(random));
        sw *= ta;
        sh *= ta;
        float ox  = crop_offset(random);
        float oy  = crop_offset(random);
        p->crop_x = (int)((isw - sw) * ox);
        p->crop_y = (int)((ish - sh) * oy);
        p->crop_w = cv_roundf(sw);
        p->crop_h = cv_roundf(sh);
    } else {
        if (padding > 0)
            throw std::invalid_argument(
                "crop_enable should not be true: when padding is defined, crop is executed by "
                "default with cropbox size equal to intput image size");
        float image_scale = scale(random);
        float hd          = horizontal_distortion(random);
        float osw = (float)out_w * hd, osh = (float)out_h;
        if (resize_short_size > 0) {
            int rw, rh;
            get_resized_short_size(in_w, in_h, resize_short_size, &rw, &rh);
            isw = (float)rw, ish = (float)rh;
        }
        float cw, ch;
        cropbox_max_proportional(isw, ish, osw, osh, &cw, &ch);
        cw *= image_scale;
        ch *= image_scale;
        float ox  = crop_offset(random);
        float oy  = crop_offset(random);
        p->crop_x = (int)((isw - cw) * ox); // cropbox_shift: float -> int truncation
        p->crop_y = (int)((ish - ch) * oy);
        p->crop_w = cv_roundf(cw);          // cv::Rect(Point2i, Size2f) -> saturate_cast
        p->crop_h = cv_roundf(ch);
    }
    if (lighting.stddev() != 0) {
        for (int i = 0; i < 3; i++) p->lighting[i] = lighting(random);
        p->n_lighting      = 3;
        p->color_noise_std = lighting.stddev();
    }
}

} // namespace aeon_hip
