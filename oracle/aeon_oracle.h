/* aeon_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of NervanaSystems/aeon's image-augmentation path (the checker
 * the HIP product is compared against).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product (aeon_amd/)
 * never links or calls it.
 *
 * Parity anchor: pinned by aeon's golden vectors
 * test/test_data/augment_output_linear_{train,eval}.bin (test/test_provider.cpp:96-261)
 * and the KATs of test/test_image.cpp (see tests/test_oracle.py).  Stages that no
 * reference fixture covers (saturation != 1, hue, lighting, 2x area path, scalar
 * row tails) follow the OpenCV-2.4 semantics restated in SURVEY.md Appendix A and
 * are "parity unpinned" -- see DESIGN.md.
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* batch_sampler (src/augment_image.hpp:343-378): sampler + sample_constraint (NaN = unset) */
typedef struct orc_batch_sampler {
    int   max_sample, max_trials;
    float scale_min, scale_max, ar_min, ar_max;
    float min_jaccard, max_jaccard, min_sample_cov, max_sample_cov, min_object_cov, max_object_cov;
} orc_batch_sampler;

/* augment::image::param_factory configuration (src/augment_image.hpp:141-246). */
typedef struct orc_aug_config {
    float scale_min, scale_max;           /* "scale"                 */
    int   angle_min, angle_max;           /* "angle"                 */
    float lighting_mean, lighting_stddev; /* "lighting"              */
    float hdist_min, hdist_max;           /* "horizontal_distortion" */
    float contrast_min, contrast_max;
    float brightness_min, brightness_max;
    float saturation_min, saturation_max;
    int   hue_min, hue_max;
    int   flip_enable, center, crop_enable, do_area_scale;
    int   resize_short_size, padding;
    float fixed_scaling_factor;           /* -1 = unset */
    int   interp;                         /* 0 LINEAR, 1 NEAREST */
    float expand_probability, expand_ratio_min, expand_ratio_max; /* make_ssd_params */
    int   n_samplers;
    orc_batch_sampler samplers[4];
} orc_aug_config;

/* augment::image::params (src/augment_image.hpp:99-119), the fields the image path reads. */
typedef struct orc_params {
    int   crop_x, crop_y, crop_w, crop_h;
    int   resize_short_size;
    int   out_w, out_h;
    int   angle, flip, padding, pad_off_x, pad_off_y;
    int   n_lighting;
    float lighting[3];
    float color_noise_std;
    float contrast, brightness, saturation;
    int   hue;
    int   interp;
    float expand_ratio;                   /* image::expand (> 1 = on) */
    int   expand_x, expand_y, expand_w, expand_h;
} orc_params;

/* image::loader configuration (src/etl_image.cpp:204-244). */
typedef struct orc_load_config {
    int    channels;       /* 1 or 3 */
    int    channel_major;  /* CHW planes vs HWC */
    int    bgr_to_rgb;
    int    out_dtype;      /* 0 uint8, 1 float32, 2 int8, 3 int16, 4 uint16, 5 int32, 6 float64 */
    int    has_mean;       /* standardize enabled */
    double mean[3];
    double stddev[3];
} orc_load_config;

/* param_factory + per-record engine.  engine_state is the minstd_rand0 state word. */
void* orc_factory_create(const orc_aug_config* cfg);
void  orc_factory_destroy(void* f);
int   orc_make_params(void* f, uint32_t* engine_state, int in_w, int in_h, int out_w, int out_h,
                      orc_params* out);
/* param_factory::make_ssd_params: boxes = n x (xmin, ymin, xmax, ymax) boundingbox::box. */
int   orc_make_ssd_params(void* f, uint32_t* engine_state, int in_w, int in_h, int out_w, int out_h,
                          const float* boxes, int n_boxes, orc_params* out);
/* batch_sampler::sample_patches of configured sampler `sampler` over n normalized boxes
 * (xmin, ymin, xmax, ymax); writes up to cap boxes to out, the count to *n_out. */
int   orc_sample_patches(void* f, int sampler, uint32_t* engine_state, const float* nboxes, int n, float* out,
                         int cap, int* n_out);
/* aeon deterministic-mode slot seeding (src/batch_decoder.cpp:47-54): n engine states. */
void  orc_seed_slots(uint32_t seed, int n, uint32_t* states);

/* geometry helpers: unbiased_round (src/util.cpp:212-239), calculate_scale (src/image.cpp:214-224),
 * cropbox_max_proportional (src/image.cpp:226-237) */
int   orc_unbiased_round(float x);
float orc_calculate_scale(int w, int h, int ow, int oh);
void  orc_cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* rw, float* rh);

/* transform_single_image (src/etl_image.cpp:146-202) -> out_h x out_w x cn uint8 HWC BGR. */
int orc_transform_image(const uint8_t* src, int w, int h, int cn, int src_stride,
                        const orc_params* p, uint8_t* out);
/* image::loader::load (src/etl_image.cpp:246-341) for the non-fixed-aspect-ratio path. */
int orc_load_image(const uint8_t* img, int w, int h, const orc_load_config* lc, void* out);
/* pixel_mask::transformer::transform (src/etl_pixel_mask.cpp:65-92), 1-channel uint8. */
int orc_transform_mask(const uint8_t* src, int w, int h, int src_stride, const orc_params* p,
                       uint8_t* out);

/* primitives, exposed for the KATs */
int  orc_resize_linear(const uint8_t* src, int sw, int sh, int sstride, int cn, uint8_t* dst,
                       int dw, int dh);
int  orc_resize_nearest(const uint8_t* src, int sw, int sh, int sstride, int cn, uint8_t* dst,
                        int dw, int dh);
int  orc_resize_cv(const uint8_t* src, int sw, int sh, int sstride, int cn, uint8_t* dst, int dw, int dh,
                   int interp);
void orc_lanczos4_coeffs(float x, float* out);
void orc_cbsjitter(uint8_t* img, int w, int h, float contrast, float brightness,
                   float saturation, int hue);
void orc_lighting(uint8_t* img, int w, int h, const float* lighting, int n, float color_noise_std);
float orc_standardize_value(int x, double mean, double stddev);
/* standardize of a uint8 canvas (fixed_aspect_ratio loader): the uint8 result of value x */
int   orc_u8_standardize_value(int x, double mean, double stddev);

/* whole-record path (transform + load) over a batch on a thread pool -- CPU baseline.
 * srcs[i] = HWC BGR uint8 image i (widths/heights per image), params[i] its params,
 * out = batch of item_bytes slots.  Returns elapsed seconds. */
/* image::rotate (src/image.cpp:53-75) over OpenCV 2.4 warpAffine: interpolate = INTER_LINEAR,
 * else INTER_NEAREST; BORDER_CONSTANT 0; output w x h x cn packed. */
int orc_rotate(const uint8_t* src, int w, int h, int cn, int stride, int angle, int interpolate, uint8_t* out);

/* transpose_regular (src/buffer_batch.cpp:186-200) as transpose_buf dispatches it (:202-244):
 * dest[c * rows + r] = src[r * cols + c], element_size 1, 2, 4 or 8.  Returns -1 otherwise. */
int orc_transpose(void* dest, const void* src, int64_t rows, int64_t cols, int element_size);

/* the CPU baseline pool's pinning (aeon's thread_affinity_map): worker t on cpus[t % n]; n = 0 unpinned */
void orc_set_affinity(const int* cpus, int n);
void orc_pool_cpus(int threads, int* out);
double orc_batch_augment(int n, const uint8_t* const* srcs, const int* widths, const int* heights,
                         const orc_params* params, const orc_load_config* lc, void* out,
                         size_t item_bytes, int threads);

/* provider_base::provide of an image + pixelmask record pair (src/provider.cpp:109-119) over a
 * batch on a thread pool: one params set per record for both -- the C5 CPU baseline. */
double orc_batch_image_mask(int n, const uint8_t* const* srcs, const uint8_t* const* masks, const int* widths,
                            const int* heights, const orc_params* params, const orc_load_config* lc,
                            void* out, size_t item_bytes, const orc_load_config* mlc, void* mout,
                            size_t mitem_bytes, int threads);

/* image::extractor::extract's JPEG decode (cv::imdecode -> libjpeg: baseline/extended Huffman,
 * ISLOW IDCT, fancy upsampling, YCbCr->RGB, emitted as BGR) -- jpeg_oracle.cpp.
 * orc_jpeg_info: frame size and component count.  orc_jpeg_decode: HWC uint8, channels 3 = BGR,
 * 1 = grayscale (Y).  Both return 0, or -1 with orc_jpeg_last_error(). */
int         orc_jpeg_info(const uint8_t* data, size_t size, int* w, int* h, int* ncomp);
int         orc_jpeg_decode(const uint8_t* data, size_t size, int channels, uint8_t* out);
const char* orc_jpeg_last_error(void);
/* the whole CPU path per record (extract -> transform -> load) over n JPEG files on a pool. */
double orc_batch_decode_augment(int n, const uint8_t* const* files, const size_t* sizes, const orc_params* params,
                                const orc_load_config* lc, void* out, size_t item_bytes, int threads);

const char* orc_last_error(void);

#ifdef __cplusplus
}
#endif
