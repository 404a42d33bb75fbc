// param_factory.cpp -- configuration parsing for augment::image::param_factory
// (aeon src/augment_image.cpp:28-105, src/interface.hpp:98-143).
#include "param_factory.hpp"

#include <algorithm>
#include <cctype>
#include <cfloat>
#include <cmath>

namespace aeon_hip {

namespace {

std::vector<double> num_array(const Json& v, const std::string& key)
{
    std::vector<double> out;
    for (const Json& e : v.array()) {
        if (!e.is_number()) throw std::invalid_argument("expected number in '" + key + "'");
        out.push_back(e.number());
    }
    return out;
}

std::vector<double> pair_of(const Json& js, const std::string& key)
{
    std::vector<double> p = num_array(js.at(key), key);
    if (p.size() < 2) throw std::invalid_argument("distribution '" + key + "' needs [a, b]");
    return p;
}

[[noreturn]] void out_of_range(const std::string& key)
{
    throw std::invalid_argument("value for '" + key + "' out of range");
}

} // namespace

// ADD_DISTRIBUTION / ADD_SCALAR parsing with aeon's validators (augment_image.hpp:208-246).
// aeon does not run verify_config on the augmentation object (augment_image.cpp:50), so
// unknown keys are ignored here too.
param_factory::param_factory(const Json& js_in)
{
    if (js_in.is_null()) return;
    if (!js_in.has("type")) throw std::invalid_argument("augmentation missing 'type'");
    const std::string type = js_in.at("type").str();
    if (type == "image") {
        const Json& js = js_in;
        auto        fpair = [&](const char* key, std::uniform_real_distribution<float>& d) {
            if (!js.has(key)) return false;
            auto p = pair_of(js, key);
            d      = std::uniform_real_distribution<float>{(float)p[0], (float)p[1]};
            return true;
        };
        auto ipair = [&](const char* key, std::uniform_int_distribution<int>& d) {
            if (!js.has(key)) return false;
            auto p = pair_of(js, key);
            d      = std::uniform_int_distribution<int>{(int)p[0], (int)p[1]};
            return true;
        };
        auto boolean = [&](const char* key, bool& v) {
            if (js.has(key)) v = js.at(key).boolean();
        };
        auto number = [&](const char* key, auto& v) {
            if (js.has(key)) v = (std::remove_reference_t<decltype(v)>)js.at(key).number();
        };
        auto string = [&](const char* key, std::string& v) {
            if (js.has(key)) v = js.at(key).str();
        };

        if (fpair("scale", scale)) {
            if (!(scale.a() >= 0 && scale.a() <= 1 && scale.b() >= 0 && scale.b() <= 1 &&
                  scale.a() <= scale.b()))
                out_of_range("scale");
        }
        if (ipair("angle", angle) && !(angle.a() <= angle.b())) out_of_range("angle");
        if (js.has("lighting")) {
            auto p   = pair_of(js, "lighting");
            lighting = std::normal_distribution<float>{(float)p[0], (float)p[1]};
        }
        if (fpair("horizontal_distortion", horizontal_distortion) &&
            !(horizontal_distortion.a() <= horizontal_distortion.b()))
            out_of_range("horizontal_distortion");
        boolean("flip_enable", flip_enable);
        boolean("center", center);
        number("resize_short_size", resize_short_size);
        string("interpolation_method", interpolation_method);
        boolean("do_area_scale", do_area_scale);
        boolean("crop_enable", crop_enable);
        number("expand_probability", expand_probability);
        boolean("fixed_aspect_ratio", fixed_aspect_ratio);
        if (js.has("mean")) mean = num_array(js.at("mean"), "mean");
        if (js.has("stddev")) stddev = num_array(js.at("stddev"), "stddev");
        number("fixed_scaling_factor", fixed_scaling_factor);
        number("padding", padding);
        string("debug_output_directory", debug_output_directory);
        if (fpair("contrast", contrast) && !(contrast.a() <= contrast.b())) out_of_range("contrast");
        if (fpair("brightness", brightness) && !(brightness.a() <= brightness.b()))
            out_of_range("brightness");
        if (fpair("saturation", saturation) && !(saturation.a() <= saturation.b()))
            out_of_range("saturation");
        if (fpair("expand_ratio", expand_ratio) &&
            !(expand_ratio.a() >= 1 && expand_ratio.a() <= expand_ratio.b()))
            out_of_range("expand_ratio");
        if (ipair("hue", hue) && !(hue.a() <= hue.b())) out_of_range("hue");
        if (js.has("batch_samplers"))
            for (const Json& b : js.at("batch_samplers").array()) batch_samplers.emplace_back(b);
        if (crop_enable && !batch_samplers.empty())
            throw std::invalid_argument(
                "'Cannot use 'batch_samplers' with 'crop_enable'. Please use only one cropping "
                "method in augmentations.");
        number("emit_constraint_min_overlap", emit_constraint_min_overlap);

        // derived (augment_image.cpp:70-85)
        if (flip_enable) flip_distribution = std::bernoulli_distribution{0.5};
        if (!center) crop_offset = std::uniform_real_distribution<float>{0.0f, 1.0f};
        if (padding > 0)
            padding_crop_offset_distribution = std::uniform_int_distribution<int>(0, padding * 2);
    }
    if (js_in.has("emit_constraint_type")) {
        std::string e = js_in.at("emit_constraint_type").str();
        std::transform(e.begin(), e.end(), e.begin(), ::tolower);
        if (!(e == "center" || e == "min_overlap" || e.empty()))
            throw std::invalid_argument("Invalid emit constraint type");
        emit_constraint_type = e;
    }
}

// ---- SSD patch sampling geometry ------------------------------------------------------------
namespace {
constexpr float kEps = 0.00001f; // nervana::epsilon (util.hpp:32)
bool normalized(float x) { return x >= 0.0f - kEps && x <= 1.0f + kEps; } // almost_equal_or_*
} // namespace

nbox::nbox(float x0, float y0, float x1, float y1) : xmin(x0), ymin(y0), xmax(x1), ymax(y1)
{
    if (!(normalized(xmin) && normalized(xmax) && normalized(ymin) && normalized(ymax)))
        throw std::invalid_argument("bounding box is not properly normalized");
}

nbox nbox::intersect(const nbox& b) const // normalized_box.cpp:75-88
{
    if (b.xmin > xmax || b.xmax < xmin || b.ymin > ymax || b.ymax < ymin) return nbox();
    return nbox(std::max(xmin, b.xmin), std::max(ymin, b.ymin), std::min(xmax, b.xmax), std::min(ymax, b.ymax));
}

float nbox::jaccard_overlap(const nbox& b) const // normalized_box.cpp:47-57
{
    const float i = intersect(b).size();
    if (i == 0.f) return 0.f;
    return i / (size() + b.size() - i);
}

float nbox::coverage(const nbox& b) const // normalized_box.cpp:59-73
{
    const float i = intersect(b).size();
    return i > 0 ? i / size() : 0.f;
}

bool sample_constraint::satisfies(const nbox& s, const std::vector<nbox>& objects) const // :404-474
{
    auto has = [](float v) { return !std::isnan(v); };
    const bool jac = has(min_jaccard_overlap) || has(max_jaccard_overlap);
    const bool sc  = has(min_sample_coverage) || has(max_sample_coverage);
    const bool oc  = has(min_object_coverage) || has(max_object_coverage);
    if (!jac && !sc && !oc) return true;
    bool found = false;
    for (const nbox& o : objects) {
        if (jac) {
            const float v = s.jaccard_overlap(o);
            if (has(min_jaccard_overlap) && v < min_jaccard_overlap) continue;
            if (has(max_jaccard_overlap) && v > max_jaccard_overlap) continue;
            found = true;
        }
        if (sc) {
            const float v = s.coverage(o);
            if (has(min_sample_coverage) && v < min_sample_coverage) continue;
            if (has(max_sample_coverage) && v > max_sample_coverage) continue;
            found = true;
        }
        if (oc) {
            const float v = o.coverage(s);
            if (has(min_object_coverage) && v < min_object_coverage) continue;
            if (has(max_object_coverage) && v > max_object_coverage) continue;
            found = true;
        }
        if (found) return true;
    }
    return found;
}

// batch_sampler / sampler / sample_constraint JSON (augment_image.hpp:262-420 config lists)
batch_sampler::batch_sampler(const Json& js)
{
    if (js.is_null()) return;
    if (js.has("max_sample")) {
        max_sample = (int)js.at("max_sample").number();
        if (max_sample < 0) out_of_range("max_sample");
    }
    if (js.has("max_trials")) max_trials = (unsigned)js.at("max_trials").number();
    if (js.has("sampler") && !js.at("sampler").is_null()) {
        const Json& sj = js.at("sampler");
        if (sj.has("scale")) {
            auto p = pair_of(sj, "scale");
            if (!(p[0] <= p[1] && p[0] > 0. && p[1] <= 1.)) out_of_range("scale");
            scale = std::uniform_real_distribution<float>{(float)p[0], (float)p[1]};
        }
        if (sj.has("aspect_ratio")) {
            auto p = pair_of(sj, "aspect_ratio");
            if (!(p[0] <= p[1] && p[0] > 0. && p[1] < FLT_MAX)) out_of_range("aspect_ratio");
            aspect_ratio = std::uniform_real_distribution<float>{(float)p[0], (float)p[1]};
        }
    }
    if (js.has("sample_constraint") && !js.at("sample_constraint").is_null()) {
        const Json& cj = js.at("sample_constraint");
        auto        f  = [&](const char* k, float& v) {
            if (cj.has(k)) v = (float)cj.at(k).number();
        };
        f("min_jaccard_overlap", constraint.min_jaccard_overlap);
        f("max_jaccard_overlap", constraint.max_jaccard_overlap);
        f("min_sample_coverage", constraint.min_sample_coverage);
        f("max_sample_coverage", constraint.max_sample_coverage);
        f("min_object_coverage", constraint.min_object_coverage);
        f("max_object_coverage", constraint.max_object_coverage);
    }
}

int param_factory::interp_code() const
{
    std::string m = interpolation_method;
    std::transform(m.begin(), m.end(), m.begin(), ::toupper);
    if (m == "LINEAR") return AEON_INTERP_LINEAR;
    if (m == "NEAREST") return AEON_INTERP_NEAREST;
    if (m == "CUBIC") return AEON_INTERP_CUBIC;
    if (m == "AREA") return AEON_INTERP_AREA;
    if (m == "LANCZOS4") return AEON_INTERP_LANCZOS4;
    throw std::invalid_argument("Provided interpolation method (" + interpolation_method +
                                " is unrecognized.");
}

int unbiased_round(float x)
{
    float i;
    float frac = std::modf(x, &i);
    int   ip   = int(i);
    int   rc;
    if (std::fabs(frac) == 0.5f) {
        if (ip % 2 == 0) {
            rc = ip;
        } else {
            rc = std::fabs(x) + 0.5;
            rc = x < 0.0 ? -rc : rc;
        }
    } else {
        rc = std::floor(std::fabs(x) + 0.5);
        rc = x < 0.0 ? -rc : rc;
    }
    return rc;
}

void get_resized_short_size(int in_w, int in_h, int target, int* ow, int* oh)
{
    float pct = static_cast<float>(target) / (float)std::min(in_h, in_w);
    *ow       = static_cast<int>(std::round((float)in_w * pct));
    *oh       = static_cast<int>(std::round((float)in_h * pct));
}

float calculate_scale(int w, int h, int ow, int oh)
{
    float s = (float)ow / (float)w;
    if ((float)h * s > oh) s = (float)oh / (float)h;
    return s;
}

void cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* rw, float* rh)
{
    float w = out_w, h = out_h;
    float s = in_w / w;
    w *= s, h *= s;
    if (h > in_h) {
        s = in_h / h;
        w *= s, h *= s;
    }
    *rw = w, *rh = h;
}

} // namespace aeon_hip
