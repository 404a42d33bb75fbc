// param_factory.cpp -- configuration parsing for augment::image::param_factory
// (aeon src/augment_image.cpp:28-105, src/interface.hpp:98-143).
#include "param_factory.hpp"

#include <algorithm>
#include <cctype>
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
        if (js.has("batch_samplers") && crop_enable && !js.at("batch_samplers").array().empty())
            throw std::invalid_argument(
                "'Cannot use 'batch_samplers' with 'crop_enable'. Please use only one cropping "
                "method in augmentations.");

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
    }
}

int param_factory::interp_code() const
{
    std::string m = interpolation_method;
    std::transform(m.begin(), m.end(), m.begin(), ::toupper);
    if (m == "LINEAR") return AEON_INTERP_LINEAR;
    if (m == "NEAREST") return AEON_INTERP_NEAREST;
    if (m == "CUBIC" || m == "AREA" || m == "LANCZOS4") return -1;
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
