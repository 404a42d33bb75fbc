/* aeon_hip.h -- C ABI of the MI355X (gfx950) image-augmentation stage for aeon.
 *
 * Drop-in boundary for aeon's decode hot path
 *   batch_decoder::process (src/batch_decoder.cpp:62-71)
 *     -> provider::image::provide (src/provider.cpp:160-184)
 *        -> image::transformer::transform_single_image (src/etl_image.cpp:146-202)
 *        -> image::loader::load (src/etl_image.cpp:246-341)
 *     -> provider::pixelmask::provide (src/provider.cpp:365-393)
 *        -> pixel_mask::transformer::transform (src/etl_pixel_mask.cpp:65-92)
 * Host code keeps decode (image::extractor::extract) and seeded parameter sampling
 * (param_factory::make_params) and calls these entry points once per decode window.
 *
 * Conventions: plain C types and pointers only; every function returns 0 on success or a
 * negative AEON_HIP_E* code, with a thread-local message in aeon_hip_last_error().
 * No C++ exception crosses this boundary.  `stream` is a hipStream_t (NULL = default stream).
 * See INTEGRATION.md for the aeon-side call sites and a ctypes binding.
 */
#ifndef AEON_HIP_H
#define AEON_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AEON_HIP_OK 0
#define AEON_HIP_EINVAL -1     /* invalid argument / configuration (aeon: std::invalid_argument) */
#define AEON_HIP_ERUNTIME -2   /* HIP runtime failure (aeon: std::runtime_error) */
#define AEON_HIP_EUNSUPPORTED -3 /* input this build refuses (e.g. arithmetic-coded / 12-bit JPEG, CMYK) */
#define AEON_HIP_EDEVICE -4    /* a kernel reported an inconsistency in its device error word */

/* output element types (aeon output_type -> cv type, src/typemap.hpp:43-52); the loader converts the
 * uint8 record with Mat::convertTo (saturating) and standardizes float / double outputs */
#define AEON_DTYPE_U8 0  /* uint8_t  (CV_8U) */
#define AEON_DTYPE_F32 1 /* float    (CV_32F) */
#define AEON_DTYPE_S8 2  /* int8_t, char (CV_8S) */
#define AEON_DTYPE_S16 3 /* int16_t  (CV_16S) */
#define AEON_DTYPE_U16 4 /* uint16_t (CV_16U) */
#define AEON_DTYPE_S32 5 /* int32_t, uint32_t (CV_32S) */
#define AEON_DTYPE_F64 6 /* double   (CV_64F) */

/* resize interpolation (image::config "interpolation_method") */
#define AEON_INTERP_LINEAR 0
#define AEON_INTERP_NEAREST 1
#define AEON_INTERP_CUBIC 2    /* cv::INTER_CUBIC (a resize pre-pass, resize_kernels.hip) */
#define AEON_INTERP_AREA 3     /* cv::INTER_AREA (2x box in the tile kernel, else a pre-pass) */
#define AEON_INTERP_LANCZOS4 4 /* cv::INTER_LANCZOS4 (a resize pre-pass) */

typedef struct aeon_hip_ctx aeon_hip_ctx;
typedef struct aeon_param_factory aeon_param_factory;

/* One decoded source image, HWC uint8 (BGR for 3 channels, OpenCV imdecode layout), living in
 * device memory at src_base + offset. Replaces cv::Mat image::decoded::get_image(0). */
typedef struct aeon_img_desc {
    uint64_t offset;   /* byte offset from the src_base passed to the batch call */
    int32_t  width;    /* cols */
    int32_t  height;   /* rows */
    int32_t  stride;   /* bytes per row (>= width*channels*elem_bytes) */
    int32_t  channels; /* 1 or 3 */
    int32_t  elem_bytes; /* bytes per channel element: 1 (CV_8U; 0 means 1) or 2 (CV_16U, the
                          * ANYDEPTH pixel masks / depth maps of etl_pixel_mask.cpp:35 and
                          * etl_depthmap.cpp:35; one channel, masks only, no rotation) */
    int32_t  reserved;
} aeon_img_desc;

/* POD mirror of augment::image::params (src/augment_image.hpp:99-119): the fields the image
 * and pixel-mask transformers read.  Produced by aeon_make_params (or by aeon itself). */
typedef struct aeon_aug_params {
    int32_t crop_x, crop_y, crop_w, crop_h; /* cropbox (cv::Rect) */
    int32_t resize_short_size;              /* 0 = off */
    int32_t out_w, out_h;                   /* output_size */
    int32_t angle;                          /* rotation (degrees, image::rotate) */
    int32_t flip;                           /* horizontal flip after photometric */
    int32_t padding, pad_off_x, pad_off_y;  /* padding + padding_crop_offset */
    int32_t n_lighting;                     /* 0 or 3 */
    float   lighting[3];                    /* PCA lighting alphas */
    float   color_noise_std;                /* lighting stddev */
    float   contrast, brightness, saturation;
    int32_t hue;
    int32_t interp;                         /* AEON_INTERP_* */
    /* image::expand (src/image.cpp:276-303; make_ssd_params, src/augment_image.cpp:246-273): with
     * expand_ratio > 1 the (rotated) record is placed at (expand_x, expand_y) of a zeroed
     * expand_w x expand_h canvas before resize_short / crop; 0 or 1 = no expand */
    float   expand_ratio;
    int32_t expand_x, expand_y, expand_w, expand_h;
} aeon_aug_params;

/* image::loader configuration (src/etl_image.cpp:204-244) plus the batch-buffer geometry of
 * fixed_buffer_map (src/buffer_batch.hpp:154-188). */
typedef struct aeon_out_desc {
    int32_t  dtype;         /* AEON_DTYPE_* */
    int32_t  channels;      /* 1 or 3 */
    int32_t  channel_major; /* 1: CHW planes, 0: HWC */
    int32_t  bgr_to_rgb;    /* swap channels 0 and 2 (3-channel only) */
    int32_t  has_mean;      /* standardize with mean/stddev (float / double output only) */
    int32_t  fixed_aspect_ratio; /* image::loader m_fixed_aspect_ratio (etl_image.cpp:258-306):
                                  * each item (its whole dtype-sized byte size) is zeroed and the
                                  * record is written at the top-left of a canvas_w x canvas_h
                                  * canvas viewed as CV_8U planes, whatever the dtype, standardized
                                  * in place as uint8 when mean/stddev are set -- aeon's layout */
    double   mean[3];
    double   stddev[3];
    uint64_t item_stride;   /* bytes between consecutive items of the batch buffer */
    int32_t  canvas_w, canvas_h; /* image::config width/height (fixed_aspect_ratio only) */
} aeon_out_desc;

/* ---- context ------------------------------------------------------------------------------ */
/* Replaces the per-loader CPU decode state; one context per GPU (hipSetDevice(device)). */
int aeon_hip_ctx_create(int device, aeon_hip_ctx** out);
int aeon_hip_ctx_destroy(aeon_hip_ctx* ctx);

/* ---- hot path ----------------------------------------------------------------------------- */
/* The per-record body of provider::image::provide after extract + make_params, for n records
 * at once: transform_single_image + image::loader::load of record i into
 * out_dev + i*out->item_stride.  Asynchronous on `stream`; src/out must stay valid until the
 * stream reaches this work.  descs/params are host arrays, consumed before return.
 * src_base / out_dev are device addresses: HBM, or pinned device-mapped host memory
 * (aeon_hip_host_alloc), which the kernels then read / store over PCIe directly (zero-copy: the
 * fastest host->host path). */
int aeon_hip_augment_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs,
                           const void* src_base, const aeon_aug_params* params,
                           const aeon_out_desc* out, void* out_dev, void* stream);

/* provider::pixelmask::provide after extract: crop -> NEAREST resize -> flip -> load, with the
 * SAME params as the image of the record (src/provider.cpp:378-391).  1-channel masks. */
int aeon_hip_mask_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs,
                        const void* src_base, const aeon_aug_params* params,
                        const aeon_out_desc* out, void* out_dev, void* stream);

/* provider::image and provider::pixelmask of the same records in one call (provider_base::provide
 * runs both with one params set per record, src/provider.cpp:109-119, 365-393): equal to
 * aeon_hip_augment_batch(descs, src_base, params, out, out_dev) followed by
 * aeon_hip_mask_batch(mask_descs, mask_src_base, params, mask_out, mask_out_dev) on `stream`.
 * When every mask is an 8-bit 1-channel record without rotation into plain uint8 items, both share
 * ONE job table (one host write, no upload launch) and run as two launches on `stream`: the image
 * tile kernel, then the masks' nearest gather reading the same table.  (A single-launch form -- the
 * masks' gather blocks taken by the image launch's workgroups after their tiles -- exists behind
 * AEON_HIP_FUSE_MASKS=1; it measured slower)  Other masks go as the two calls. */
int aeon_hip_augment_pair_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs,
                                const void* src_base, const aeon_img_desc* mask_descs,
                                const void* mask_src_base, const aeon_aug_params* params,
                                const aeon_out_desc* out, void* out_dev,
                                const aeon_out_desc* mask_out, void* mask_out_dev, void* stream);

/* depthmap::extractor -> transformer -> loader (src/etl_depthmap.cpp:30-134) after extract: the
 * pixel-mask transform (rotate nearest -> crop -> NEAREST resize -> flip) and a plain
 * convert_mix_channels load (no fixed_aspect_ratio canvas).  aeon's provider_factory does not
 * construct depth maps (src/provider.cpp:43-99); this is the entry a depthmap provider calls. */
int aeon_hip_depthmap_batch(aeon_hip_ctx* ctx, int n, const aeon_img_desc* descs,
                            const void* src_base, const aeon_aug_params* params,
                            const aeon_out_desc* out, void* out_dev, void* stream);

/* batch_major=false output layout: fixed_buffer_map::copy(..., transpose=true) ->
 * transpose_buf (src/buffer_batch.cpp:186-244, 251-280; called per batch by
 * batch_iterator_fbm::filler, src/batch_iterator.cpp:125-136):
 *   dst[c * rows + r] = src[r * cols + c]
 * for a rows x cols matrix of element_size-byte elements (rows = batch size, cols = elements
 * per item).  element_size 1, 2, 4 or 8; src and dst are device buffers that must not overlap.
 * Async on `stream`. */
int aeon_hip_transpose_batch(aeon_hip_ctx* ctx, const void* src_dev, void* dst_dev, int64_t rows,
                             int64_t cols, int element_size, void* stream);

/* ---- decode (image::extractor::extract, src/etl_image.cpp:83-99) ---------------------------- */
/* JPEG frame header: width, height, component count (1 or 3).  Host only, no context needed. */
int aeon_jpeg_info(const void* data, size_t size, int* width, int* height, int* components);
/* The host half of the JPEG stage alone (headers, Huffman tables, every scan's entropy decoding into
 * the sparse coefficient stream aeon_hip_decode_jpeg_batch uploads), on the calling thread, no device:
 * the stream's block / non-zero value counts and an FNV-1a hash of it.  For robustness tests of the
 * untrusted-input parser (sanitizer builds, malformed-file corpora).  Same error codes as the batch
 * decode. */
int aeon_jpeg_entropy_decode(const void* data, size_t size, int* width, int* height, int* components,
                             int64_t* n_blocks, int64_t* n_values, uint64_t* hash);
/* The host work aeon_hip_decode_jpeg_batch does for one file, on the calling thread, no device: a
 * sequential file with one scan of every component gets its headers parsed and its entropy-coded
 * bytes unstuffed for the GPU Huffman decoder (*gpu_entropy = 1); any other (progressive,
 * multi-scan) is entropy-decoded into the sparse stream (*gpu_entropy = 0).  *staged_bytes: what it
 * stages for the H2D.  For timing the host side of the stage per file. */
int aeon_jpeg_host_stage(const void* data, size_t size, int* gpu_entropy, int64_t* staged_bytes);
/* cv::imdecode(CV_LOAD_IMAGE_COLOR / GRAYSCALE) of n JPEG files (baseline / extended sequential /
 * progressive Huffman, 8-bit, 1 or 3 components) as libjpeg decodes them (ISLOW IDCT, fancy upsampling),
 * into device memory: record i as HWC uint8 (BGR if descs[i].channels == 3, the Y component if 1)
 * at dst_base + descs[i].offset with descs[i].stride bytes per row; descs[i].width/height must be
 * the file's (aeon_jpeg_info).  Headers are parsed on the context's host pool; sequential files with
 * one scan of every component are Huffman-decoded on the GPU (their unstuffed entropy-coded bytes go
 * up), the others on the pool (their sparse coefficients go up), all in one H2D; the Huffman, IDCT /
 * upsampling / colour conversion kernels run on `stream`.  Corrupt entropy-coded data of a
 * GPU-decoded file is reported by aeon_hip_synchronize (AEON_HIP_EDEVICE).  The files may be released when the call returns; dst must stay valid until the stream
 * reaches the work.  Arithmetic-coded / lossless / 12-bit / CMYK files: AEON_HIP_EUNSUPPORTED. */
int aeon_hip_decode_jpeg_batch(aeon_hip_ctx* ctx, int n, const void* const* data, const size_t* sizes,
                               const aeon_img_desc* descs, void* dst_base, void* stream);

/* Wait for `stream` and check the device error word of the calls made on it (each stream has its own
 * word, so a window's check never reads or clears what another stream's kernels set):
 * AEON_HIP_EDEVICE (the word cleared) when a kernel flagged an inconsistency -- an LDS footprint the host sized too small, a dynamic-tail counter
 * not reset by an earlier launch, a rotation source box over its LDS.  None is expected. */
int aeon_hip_synchronize(aeon_hip_ctx* ctx, void* stream);

/* Streams: the context records one completion event per few calls on the stream of the calls (its ring
 * slots are reused after it), so a stream the calls ran on must stay valid until aeon_hip_synchronize or
 * aeon_hip_release_stream has been called on it (or the context is destroyed).  aeon_hip_release_stream:
 * the caller is about to destroy `stream` -- the pending completion event is recorded on it now and the
 * context keeps no reference to it.  No wait. */
int aeon_hip_release_stream(aeon_hip_ctx* ctx, void* stream);

/* ---- measurement ---------------------------------------------------------------------------- */
/* every > 0: the kernel launches of one augment/mask call in `every` -- the every-th, 2*every-th,
 * ... call after this one, so never the first launch after an idle GPU -- are bracketed by HIP
 * events on their own stream (an event pair costs GPU time between launches, so benchmarks
 * sample); 0 disables timing. */
int aeon_hip_set_timing(aeon_hip_ctx* ctx, int every);
/* Drain the timers: per kernel kind [0]=augment (final), [1]=contrast statistics,
 * [2]=pre-passes (resize_short, CUBIC / AREA / LANCZOS4 resize, 2x-area ahead of photometric),
 * [3]=JPEG IDCT + colour kernels of aeon_hip_decode_jpeg_batch (bytes: decoded pixels): total ms,
 * total algorithmic bytes, launches.  The arrays hold `kinds` entries (AEON_HIP_TIMER_KINDS = all;
 * fewer are filled, more are left alone).  Resets the totals of every kind. */
#define AEON_HIP_TIMER_KINDS 4
int aeon_hip_kernel_times(aeon_hip_ctx* ctx, int kinds, double* ms, double* bytes, long* count);

/* ---- augmentation parameters (host) ------------------------------------------------------- */
/* augment::image::param_factory(json) (src/augment_image.cpp:28-89) from the JSON text of the
 * "augmentation" object ({"type": "image", ...}).  Validators as aeon; like aeon (which skips
 * verify_config here, src/augment_image.cpp:50) unknown keys are ignored. */
int aeon_param_factory_create(const char* aug_json, aeon_param_factory** out);
int aeon_param_factory_destroy(aeon_param_factory* f);
/* param_factory::make_params (src/augment_image.cpp:107-230) drawing from the minstd_rand0
 * engine whose state word is *engine_state (updated in place).  Calls on one factory are
 * serialised internally, but the lighting normal_distribution caches its second draw inside the
 * factory (as aeon's shared, mutable one does), so reproducible lighting needs one calling thread
 * making the calls in record order -- aeon's own deterministic order. */
int aeon_make_params(aeon_param_factory* f, uint32_t* engine_state, int in_w, int in_h,
                     int out_w, int out_h, aeon_aug_params* out);
/* param_factory::make_ssd_params (src/augment_image.cpp:232-301): make_params, then expand
 * (expand_ratio / expand_probability) and -- crop_enable false -- a patch from the configured
 * batch_samplers (sampler scale / aspect_ratio, sample_constraint jaccard / coverage bounds, max_sample,
 * max_trials; src/augment_image.cpp:303-586) as the cropbox of the expanded image.  boxes: n_boxes
 * object boxes (xmin, ymin, xmax, ymax; boundingbox::box pixel coordinates, xmax inclusive), may be
 * NULL when n_boxes is 0.  Same engine and draw order as aeon, so the same state gives aeon's params. */
int aeon_make_ssd_params(aeon_param_factory* f, uint32_t* engine_state, int in_w, int in_h, int out_w, int out_h,
                         const float* boxes, int n_boxes, aeon_aug_params* out);

/* PNG decode -- image::extractor::extract / pixel_mask::extractor::extract on PNG files
 * (src/etl_image.cpp:83-99, src/etl_pixel_mask.cpp:30-53: cv::imdecode over libpng), on the host.
 * Modes: AEON_PNG_BGR8 = CV_LOAD_IMAGE_COLOR (8-bit BGR), AEON_PNG_GRAY8 = CV_LOAD_IMAGE_GRAYSCALE,
 * AEON_PNG_ANYDEPTH = CV_LOAD_IMAGE_ANYDEPTH (gray at the file's depth: 16-bit files give native
 * uint16 samples).  aeon_png_info: size, bit depth and PNG colour type from the header.
 * aeon_decode_png writes height rows of `stride` bytes to dst and the element size (1 or 2) to
 * *elem_bytes (may be NULL). */
#define AEON_PNG_BGR8     0
#define AEON_PNG_GRAY8    1
#define AEON_PNG_ANYDEPTH 2
int aeon_png_info(const void* data, size_t size, int* width, int* height, int* bit_depth, int* color_type);
int aeon_decode_png(const void* data, size_t size, int mode, void* dst, size_t stride, int* elem_bytes);

/* batch_sampler::sample_patches (src/augment_image.cpp:567-586) of the factory's batch_samplers[sampler]
 * over n normalized object boxes (xmin, ymin, xmax, ymax in [0, 1]) -- what aeon's tests call as
 * factory.m_batch_samplers[i].sample_patches (test/test_augmentation.cpp:347-443).  Writes up to cap
 * boxes to out (4 floats each) and the number of samples found to *n_out. */
int aeon_batch_sample_patches(aeon_param_factory* f, int sampler, uint32_t* engine_state, const float* nboxes, int n,
                              float* out, int cap, int* n_out);

/* batch_decoder deterministic mode (src/batch_decoder.cpp:47-54): slot engine state words. */
int aeon_seed_slots(uint32_t seed, int n, uint32_t* states);

/* Host geometry helpers make_params is built on (exported for callers that derive their own
 * cropboxes, e.g. a localization provider, and for the reference's known-answer tests):
 *   nervana::unbiased_round (src/util.cpp:212-239)
 *   image::calculate_scale (src/image.cpp:214-224)
 *   image::cropbox_max_proportional (src/image.cpp:226-237) */
int aeon_unbiased_round(float x, int64_t* out);
int aeon_calculate_scale(int width, int height, int output_width, int output_height, float* scale);
int aeon_cropbox_max_proportional(float in_w, float in_h, float out_w, float out_h, float* res_w,
                                  float* res_h);

/* ---- decode stage: provider_factory + batch_decoder (host C++ above the kernels) --------------
 * aeon_decoder = batch_decoder (src/batch_decoder.cpp:24-99) over provider_factory::create
 * (src/provider_factory.cpp:24-51) with "image" / "pixelmask" ETL providers.  config_json is the
 * aeon loader configuration ({"batch_size", "random_seed", "node_id", "cpu_list", "etl": [...],
 * "augmentation": [...]}, src/loader.hpp:50-109; unknown keys are rejected like verify_config).
 * Records arrive decoded (image::extractor::extract stays with the caller). */
typedef struct aeon_decoder aeon_decoder;

/* One decoded element of a record: HWC uint8 (BGR) pixels in host memory. */
typedef struct aeon_record_elem {
    const void* data;
    int32_t     width, height, channels;
    int32_t     stride; /* bytes per row; 0 = width*channels */
} aeon_record_elem;

int aeon_decoder_create(const char* config_json, int device, aeon_decoder** out);
int aeon_decoder_destroy(aeon_decoder* d);
/* provider_interface::get_output_shapes (src/provider_interface.hpp:61-65) */
int aeon_decoder_output_count(aeon_decoder* d, int* count);
int aeon_decoder_output_info(aeon_decoder* d, int index, char* name, size_t name_cap, int64_t* shape,
                             int* ndim, size_t* item_bytes, int* dtype);
/* One decode window: n records x input_count elements (row-major in elems).  outputs[k] holds
 * n items of output k (host memory, or device memory when outputs_on_device).  Returns when
 * the window is complete (batch_decoder::filler, src/batch_decoder.cpp:73-99). */
int aeon_decoder_decode(aeon_decoder* d, int n, const aeon_record_elem* elems, void* const* outputs,
                        int outputs_on_device, void* stream);
/* The host half of a window alone (no GPU): batch_decoder::process's make_params for n records
 * (src/batch_decoder.cpp:62-71, augment_image.cpp:107-230) with the decoder's slot engines, which
 * advance as in a real window; params[i] = record i's params.  serial = 1 draws in record order on
 * the calling thread, 0 on the decoder's pool (identical params).  Only elems' sizes are read. */
int aeon_decoder_draw_params(aeon_decoder* d, int n, const aeon_record_elem* elems, aeon_aug_params* params,
                             int serial);
/* A record element as aeon's encoded_record holds it (src/buffer_batch.hpp:45-152): an encoded
 * JPEG file (width == 0: data/size, decoded by the JPEG stage with the provider's channel count),
 * or -- width > 0 -- decoded HWC uint8 pixels as in aeon_record_elem (pixel masks must be). */
typedef struct aeon_encoded_elem {
    const void* data;
    size_t      size;
    int32_t     width, height, channels;
    int32_t     stride; /* decoded pixels only; 0 = width*channels */
} aeon_encoded_elem;

/* As aeon_decoder_decode, from encoded records: extract (JPEG) + transform + load per record. */
int aeon_decoder_decode_encoded(aeon_decoder* d, int n, const aeon_encoded_elem* elems, void* const* outputs,
                                int outputs_on_device, void* stream);
/* Double-buffered decode windows (async_manager's two containers, src/async_manager.hpp:91-114,
 * 162-204): submit returns once the window's input bytes are consumed (params drawn, pixels staged,
 * JPEGs entropy-decoded) with its copies and kernels queued on the decoder's own stream; at most two
 * windows are in flight, and outputs[k] must stay valid until aeon_decoder_wait returns for that
 * window (windows complete in submission order).  Host outputs should be pinned
 * (aeon_hip_host_alloc) for the D2H to overlap the next window. */
int aeon_decoder_submit(aeon_decoder* d, int n, const aeon_encoded_elem* elems, void* const* outputs,
                        int outputs_on_device);
int aeon_decoder_wait(aeon_decoder* d);
/* The decode pool's CPU pinning (thread_pool.hpp:133-138 + util.cpp:337-373).
 * aeon_thread_affinity_map: nervana::get_thread_affinity_map -- AEON_CPU_LIST, else cpu_list ("0-3,8"),
 * else hc - min(2, hc/8) CPUs: the first ones of the process's affinity mask (aeon: iota from 0, which is
 * the same list on an unrestricted host).  Writes up to cap ids, the map's length to *count.
 * aeon_decoder_pool_size / aeon_decoder_pool_cpus: the decoder's workers; for worker i, the CPU of the map
 * it was pinned to (*map_cpu, -1 = none) and the CPUs its own sched_getaffinity reported after pinning
 * (a CPU outside the process's cpuset cannot be pinned to: that worker reports the process mask). */
int aeon_thread_affinity_map(const char* cpu_list, int* cpus, int cap, int* count);
int aeon_decoder_pool_size(aeon_decoder* d, int* workers);
int aeon_decoder_pool_cpus(aeon_decoder* d, int worker, int* map_cpu, int* cpus, int cap, int* count);
const char* aeon_decoder_last_error(void);

/* manifest_file node slicing (src/manifest_file.cpp:278-295): the record indices of node
 * node_id of node_count (indices may be NULL to query *count). */
int aeon_manifest_node_slice(int64_t record_count, int batch_size, int node_id, int node_count,
                             int64_t* indices, int64_t* count);

/* ---- the aeon-side drop-in: provide() stages, post_process() flushes ---------------------------
 * What provider::image / provider::pixelmask hold.  aeon's batch_decoder::filler runs
 * provide(idx, record, out_buf) for a decode window on its pool (src/batch_decoder.cpp:62-99) and, with
 * the one-line change, post_process(out_buf) once per batch of the window; provider_base forwards
 * post_process to each ETL provider (src/provider.hpp:64-76 gains the override).
 *   aeon_hip_stager_stage (from provide(), any pool thread, concurrently): record idx of the batch whose
 *     buffer is batch_out (out_buf[name]->get_item(0): the staging key) -- its decoded pixels (HWC,
 *     copied into pinned memory before the call returns) and its augment::image::params.
 *   aeon_hip_stager_launch (from post_process(), the filler thread): the first launch after a window's
 *     stages launches the WHOLE window on the window's own stream -- one H2D per pinned staging chunk,
 *     one augment (or pixel-mask) launch over every staged record of every batch, a D2H into each batch
 *     buffer (pinned, device-mapped batch buffers are stored into directly; AEON_STAGER_DEVICE_OUT:
 *     batch_out is device memory) -- and returns without waiting; later launches of the window's other
 *     batches only mark them.  A batch must hold idx 0..n-1.
 *   aeon_hip_stager_wait (from the consumer, batch_iterator_fbm::filler, src/batch_iterator.cpp:109-142,
 *     before it swaps or copies a batch out of the decoded container): returns once batch_out is
 *     complete.  stager may be NULL: the library finds the stager that launched batch_out (the consumer
 *     knows the buffers, not the providers); a buffer no stager launched (another ETL's, or one already
 *     waited for) returns 0 at once.  The window's last wait surfaces the device error word.
 *   aeon_hip_stager_flush: launch + wait for batch_out (a post_process that returns a finished batch).
 * Two windows are kept (aeon's async_manager, src/async_manager.hpp:162-204, has two containers): the
 * stages of window k+1 go to the other one while window k's copies and kernels run; staging a third
 * window while the first was never waited for completes and drops that first one.
 * Images: aeon_hip_augment_batch semantics; masks (AEON_STAGER_MASK): aeon_hip_mask_batch, staged with
 * the record's image params (provider.cpp:378-391).  Errors: AEON_HIP_E* codes,
 * aeon_hip_stager_last_error(); a window whose launch fails is dropped whole. */
typedef struct aeon_hip_stager aeon_hip_stager;
#define AEON_STAGER_IMAGE      0
#define AEON_STAGER_MASK       1
#define AEON_STAGER_DEVICE_OUT 0x100 /* or-ed into kind: batch buffers are device memory */
int aeon_hip_stager_create(aeon_hip_ctx* ctx, int kind, const aeon_out_desc* out, int batch_size,
                           aeon_hip_stager** stager);
int aeon_hip_stager_destroy(aeon_hip_stager* stager);
int aeon_hip_stager_stage(aeon_hip_stager* stager, void* batch_out, int idx, const void* pixels, int width,
                          int height, int stride, int channels, int elem_bytes, const aeon_aug_params* params);
int aeon_hip_stager_launch(aeon_hip_stager* stager, void* batch_out);
int aeon_hip_stager_wait(aeon_hip_stager* stager, void* batch_out);
int aeon_hip_stager_flush(aeon_hip_stager* stager, void* batch_out);
const char* aeon_hip_stager_last_error(void);

/* ---- host staging (replaces the dead cuMemAllocHost branch, src/buffer_batch.cpp:150-186) -- */
int aeon_hip_host_alloc(size_t bytes, void** out);
int aeon_hip_host_free(void* p);

/* Diagnostics: the device address ranges [lo, hi) of every uncached job-table block this process
 * allocated (stage.cpp grow_vram; they are pooled, never freed: DESIGN.md §8), up to cap pairs into
 * ranges; *n = how many there are.  Lets a test that finds lost writes say whether they lie inside one. */
int aeon_hip_debug_uncached_blocks(uint64_t* ranges, int cap, int* n);

const char* aeon_hip_last_error(void);
const char* aeon_hip_version(void);

#ifdef __cplusplus
}
#endif

#endif /* AEON_HIP_H */
