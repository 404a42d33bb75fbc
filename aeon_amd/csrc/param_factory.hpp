// param_factory.hpp -- augment::image::param_factory for the HIP stage (host C++).
//
// Same configuration keys, validators, distributions and RNG draw order as aeon's
// src/augment_image.hpp:125-249 / src/augment_image.cpp:28-230, so a record drawn from the
// same minstd_rand0 state gets the same params as in aeon.  Parameter sampling stays on the
// host (µs per record); the pixel work it parameterises runs on the GPU.
#pragma once
#include <cmath>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/aeon_hip.h"
#include "json.hpp"

namespace aeon_hip {

// normalized_box::box (src/normalized_box.hpp:24-67): coordinates in [0, 1] (within aeon's 1e-5
// epsilon, src/util.cpp:246-254), width = xmax - xmin.  Constructing an improperly normalized box
// throws std::invalid_argument, as aeon's constructor does.
struct nbox {
    float xmin = 0, ymin = 0, xmax = 0, ymax = 0;
    nbox() = default;
    nbox(float x0, float y0, float x1, float y1);
    float size() const { return (xmax < xmin || ymax < ymin) ? 0.0f : (xmax - xmin) * (ymax - ymin); }
    nbox  intersect(const nbox& b) const;
    float jaccard_overlap(const nbox& b) const;
    float coverage(const nbox& b) const;
};

// sample_constraint (src/augment_image.cpp:404-474): NaN = bound not configured
struct sample_constraint {
    float min_jaccard_overlap = NAN, max_jaccard_overlap = NAN;
    float min_sample_coverage = NAN, max_sample_coverage = NAN;
    float min_object_coverage = NAN, max_object_coverage = NAN;
    bool  satisfies(const nbox& sampled, const std::vector<nbox>& objects) const;
};

// sampler + batch_sampler (src/augment_image.cpp:355-402, 556-586)
struct batch_sampler {
    int                                           max_sample = -1;
    unsigned                                      max_trials = 100;
    mutable std::uniform_real_distribution<float> scale{1.0f, 1.0f}, aspect_ratio{1.0f, 1.0f};
    sample_constraint                             constraint;
    explicit batch_sampler(const Json& js);
    template <typename URNG>
    nbox sample_patch(URNG& random) const;
    template <typename URNG>
    void sample_patches(URNG& random, const std::vector<nbox>& objects, std::vector<nbox>& out) const;
};

class param_factory {
public:
    explicit param_factory(const Json& js);

    // src/augment_image.cpp:107-230
    template <typename URNG>
    void make_params(URNG& random, int in_w, int in_h, int out_w, int out_h, aeon_aug_params* p) const;

    // make_params of one record of a decode window drawn out of order (the decoder's parallel draw):
    // `lighting`'s cache (below) is the only state one record's draw hands to the next, and its
    // availability at record i's entry is known up front (every record makes exactly three normal
    // draws, each toggling it), so record i draws with its own engine as if the cache held
    // `entry_avail`; a cached first value is left as NaN for the window's in-order fix-up
    // (light_fixup), and a value the record leaves cached is returned in *exit_saved.
    template <typename URNG>
    void make_params_split(URNG& random, int in_w, int in_h, int out_w, int out_h, bool entry_avail,
                           aeon_aug_params* p, float* exit_saved) const;
    bool  lighting_on() const { return lighting.stddev() != 0; }
    bool  light_avail() const { return m_light_avail; }
    float light_saved() const { return m_light_saved; }
    void  set_light_state(bool avail, float saved) const { m_light_avail = avail, m_light_saved = saved; }

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

    int interp_code() const; // AEON_INTERP_*

private:
    // std::normal_distribution<float>'s cache, restated (libstdc++ bits/random.tcc: the polar
    // method makes a pair, returns one value and keeps the other for the next call): lighting
    // draws go through light_draw, which makes each pair with a fresh distribution of the same
    // param -- the pair depends only on the engine -- so the cache can be read, set and handed
    // across records (make_params_split).
    mutable bool  m_light_avail = false;
    mutable float m_light_saved = 0.f;
    template <typename URNG>
    float light_draw(URNG& random) const
    {
        if (m_light_avail) {
            m_light_avail = false;
            return m_light_saved;
        }
        std::normal_distribution<float> d(lighting.param());
        const float y = d(random);
        m_light_saved = d(random); // the pair's cached second value: no engine draw
        m_light_avail = true;
        return y;
    }
    template <typename URNG>
    void make_geometry(URNG& random, int in_w, int in_h, int out_w, int out_h, aeon_aug_params* p) const;

public:

    // src/augment_image.cpp:232-301 (boxes: n x (xmin, ymin, xmax, ymax) boundingbox::box)
    template <typename URNG>
    void make_ssd_params(URNG& random, int in_w, int in_h, int out_w, int out_h, const float* boxes, int n_boxes,
                         aeon_aug_params* p) const;

    std::vector<batch_sampler>                    batch_samplers;
    mutable std::uniform_real_distribution<float> expand_distribution{0.0f, 1.0f};
    std::string                                   emit_constraint_type;
    float                                         emit_constraint_min_overlap = 0.0f;
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
    make_geometry(random, in_w, in_h, out_w, out_h, p);
    if (lighting.stddev() != 0) { // the last draws of make_params (augment_image.cpp:218-225)
        for (int i = 0; i < 3; i++) p->lighting[i] = light_draw(random);
        p->n_lighting      = 3;
        p->color_noise_std = lighting.stddev();
    }
}

template <typename URNG>
void param_factory::make_params_split(URNG& random, int in_w, int in_h, int out_w, int out_h, bool entry_avail,
                                      aeon_aug_params* p, float* exit_saved) const
{
    make_geometry(random, in_w, in_h, out_w, out_h, p);
    if (lighting.stddev() == 0) return;
    std::normal_distribution<float> d(lighting.param());
    if (entry_avail) { // cached value first (light_fixup), then one pair from this engine: cache empty
        p->lighting[0] = NAN;
        p->lighting[1] = d(random);
        p->lighting[2] = d(random);
    } else { // two pairs from this engine; the second pair's other value stays cached
        p->lighting[0] = d(random);
        p->lighting[1] = d(random);
        p->lighting[2] = d(random);
        *exit_saved    = d(random);
    }
    p->n_lighting      = 3;
    p->color_noise_std = lighting.stddev();
}

// make_params up to (not including) the lighting draws
template <typename URNG>
void param_factory::make_geometry(URNG& random, int in_w, int in_h, int out_w, int out_h,
                                  aeon_aug_params* p) const
{
    *p            = aeon_aug_params{};
    p->expand_ratio = 1.0f; // augment::image::params default (augment_image.hpp:99): make_params leaves it
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
}

// sampler::sample_patch (src/augment_image.cpp:355-384): float scale, aspect ratio bounded by
// scale^2 (pow in double, then float), box of scale * sqrt(ar) x scale / sqrt(ar) at a uniform offset
template <typename URNG>
nbox batch_sampler::sample_patch(URNG& random) const
{
    const float s      = scale(random);
    const float min_ar = std::max<float>(aspect_ratio.min(), std::pow(s, 2.));
    const float max_ar = std::min<float>(aspect_ratio.max(), 1 / std::pow(s, 2.));
    const float ar     = std::uniform_real_distribution<float>(min_ar, max_ar)(random);
    const float bw = s * std::sqrt(ar), bh = s / std::sqrt(ar);
    const float w_off  = std::uniform_real_distribution<float>(0.f, 1.f - bw)(random);
    const float h_off  = std::uniform_real_distribution<float>(0.f, 1.f - bh)(random);
    return nbox(w_off, h_off, w_off + bw, h_off + bh);
}

// batch_sampler::sample_patches (src/augment_image.cpp:568-586)
template <typename URNG>
void batch_sampler::sample_patches(URNG& random, const std::vector<nbox>& objects, std::vector<nbox>& out) const
{
    int found = 0;
    for (unsigned i = 0; i < max_trials; ++i) {
        if (max_sample != -1 && found >= max_sample) break;
        const nbox sampled = sample_patch(random);
        if (constraint.satisfies(sampled, objects)) {
            ++found;
            out.push_back(sampled);
        }
    }
}

template <typename URNG>
void param_factory::make_ssd_params(URNG& random, int in_w, int in_h, int out_w, int out_h, const float* boxes,
                                    int n_boxes, aeon_aug_params* p) const
{
    make_params(random, in_w, in_h, out_w, out_h, p);
    p->out_w = out_w, p->out_h = out_h; // "use warping"
    float     ratio   = expand_ratio(random);
    const bool enabled = expand_distribution(random) < expand_probability;
    if (ratio < 1.) throw std::invalid_argument("Expand ratio must be greater than 1.");
    int ox = 0, oy = 0, ew = in_w, eh = in_h;
    if (enabled) {
        const float fw = ratio * (float)(size_t)in_w, fh = ratio * (float)(size_t)in_h;
        ew = (int)std::floor(fw), eh = (int)std::floor(fh);
        const float mw = fw - (float)(size_t)in_w, mh = fh - (float)(size_t)in_h;
        const float w_off = expand_distribution(random) * mw;
        const float h_off = expand_distribution(random) * mh;
        ox = (int)std::floor(w_off), oy = (int)std::floor(h_off);
    } else {
        ratio = 1.0f;
    }
    p->expand_ratio = ratio, p->expand_x = ox, p->expand_y = oy, p->expand_w = ew, p->expand_h = eh;
    // boundingbox::expand then normalize (boundingbox.cpp:88-105, 150-163)
    std::vector<nbox> objects;
    for (int i = 0; i < n_boxes; i++) {
        const float* b = boxes + 4 * i;
        if (b[2] + ox > ew || b[3] + oy > eh) throw std::invalid_argument("Invalid parameters to expand boundingbox");
        const float x0 = b[0] + ox, y0 = b[1] + oy, x1 = b[2] + ox, y1 = b[3] + oy;
        objects.emplace_back(x0 / ew, y0 / eh, (x1 + 1) / ew, (y1 + 1) / eh);
    }
    if (!crop_enable) {
        // param_factory::sample_patch (src/augment_image.cpp:303-322)
        std::vector<nbox> samples;
        for (const batch_sampler& bs : batch_samplers) bs.sample_patches(random, objects, samples);
        nbox patch(0, 0, 1, 1);
        if (!samples.empty()) patch = samples[std::uniform_int_distribution<int>(0, (int)samples.size() - 1)(random)];
        // unnormalize (normalized_box.hpp:59-63) -> boundingbox rect() (box.hpp:53-57)
        const float x0 = patch.xmin * (float)ew, y0 = patch.ymin * (float)eh;
        const float x1 = patch.xmax * (float)ew - 1, y1 = patch.ymax * (float)eh - 1;
        p->crop_x = (int)std::round(x0), p->crop_y = (int)std::round(y0);
        p->crop_w = (int)std::round(x1 - x0 + 1), p->crop_h = (int)std::round(y1 - y0 + 1);
    }
}

} // namespace aeon_hip
