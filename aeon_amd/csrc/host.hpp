// host.hpp -- aeon's provider plugin surface and decode stage for the HIP image path (host C++).
//
// Mirrors, with the same names and argument meaning:
//   provider_interface       src/provider_interface.hpp:32-85  (post_process = the GPU flush)
//   provider_factory::create src/provider_factory.cpp:24-51
//   provider::image          src/provider.cpp:145-184          (etl type "image")
//   provider::pixelmask      src/provider.cpp:353-393          (etl type "pixelmask")
//   image::config            src/etl_image.hpp:56-96, etl_image.cpp:25-65
//   batch_decoder            src/batch_decoder.cpp:24-99        (thread pool + deterministic slots)
//   thread_pool              src/thread_pool.hpp:82-175         (dynamic atomic task counter)
//   manifest node slicing    src/manifest_file.cpp:278-295
// Records arrive as encoded JPEG files (image::extractor::extract's cv::imdecode runs in the
// JPEG stage: host Huffman + GPU IDCT/colour, jpeg_host.cpp) or as decoded HWC uint8 pixels (staged
// into pinned memory by the pool).  One flush per decode window runs the HIP kernels; windows are
// double-buffered like async_manager's two containers (submit / wait).
#pragma once
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/aeon_hip.h"
#include "json.hpp"
#include "param_factory.hpp"

namespace aeon_hip {

// typemap.hpp output_type (the types this stage writes)
struct output_type {
    std::string name;
    size_t      size  = 1;
    int         dtype = AEON_DTYPE_U8;
    explicit output_type(const std::string& n = "uint8_t");
    static bool is_valid_type(const std::string& n);
};

struct shape_type {
    std::vector<size_t>      shape;
    std::vector<std::string> names;
    output_type              otype;
    size_t                   byte_size() const;
};

// image::config
struct image_config {
    uint32_t    height = 0, width = 0;
    std::string output_type_name = "uint8_t";
    bool        bgr_to_rgb = false, channel_major = true;
    uint32_t    channels = 3;
    std::string name;
    shape_type  shape;
    explicit image_config(const Json& js);
};

// An element of a record: an encoded JPEG file (size > 0; width/height/channels filled in from
// its header by the decoder) or decoded HWC uint8 pixels (what image::extractor::extract returns).
struct decoded_element {
    const uint8_t* data = nullptr;
    int            width = 0, height = 0, channels = 0, stride = 0;
    size_t         size    = 0;     // encoded bytes
    bool           encoded = false; // JPEG file: decoded on the device (jpeg_host.cpp)
    int            png_mode   = -1; // PNG file: AEON_PNG_* decode on the host while staging
    int            elem_bytes = 1;  // bytes per sample (2: a 16-bit mask / depth map)
};

// Per-window staging shared by the providers (filled concurrently by the pool threads).
struct decode_window {
    int                                       n = 0;
    std::vector<std::vector<aeon_img_desc>>   descs;  // [provider][record]
    std::vector<std::vector<aeon_aug_params>> params; // [provider][record]
    std::vector<std::vector<size_t>>          offset; // [provider][record] in the pinned arena
    uint8_t*                                  arena = nullptr;
};

// augmentation shared by the ETL providers of one record (provider.cpp:109-119)
struct augmentation {
    bool            has = false;
    aeon_aug_params image{};
};

class provider_interface {
public:
    provider_interface(Json js, size_t input_count) : m_js(std::move(js)), m_input_count(input_count) {}
    virtual ~provider_interface() = default;

    size_t                                                  get_input_count() const { return m_input_count; }
    const std::vector<std::pair<std::string, shape_type>>& get_output_shapes() const { return m_output_shapes; }
    const shape_type&                                       get_output_shape(const std::string& name) const;
    const std::vector<std::string>&                         get_buffer_names();
    const Json&                                             get_config() const { return m_js; }

protected:
    std::vector<std::pair<std::string, shape_type>> m_output_shapes;
    std::vector<std::string>                        m_buffer_names;
    Json                                            m_js;
    size_t                                          m_input_count = 0;
};

class thread_pool;

// One record's share of a parallel window draw (param_factory::make_params_split): the lighting
// cache state it starts from, and the value it leaves cached.
struct light_split {
    bool  entry_avail = false;
    float exit_saved  = 0.f;
};

// One ETL element provider of the HIP stage (provider::image / provider::pixelmask).
class etl_provider {
public:
    virtual ~etl_provider() = default;
    // host half of provide(): params for record idx (shared through aug) + its descriptor; with ls,
    // the record is drawn out of order (provider_base::draw_window)
    virtual void provide(int idx, const decoded_element& in, augmentation& aug, std::minstd_rand0& random,
                         aeon_aug_params& params, light_split* ls = nullptr) const = 0;
    virtual const param_factory& factory() const = 0;
    virtual bool               is_mask() const = 0;
    virtual const shape_type&  shape() const = 0;
    virtual const std::string& buffer_name() const = 0;
    virtual aeon_out_desc      out_desc() const = 0;
};

class provider_base : public provider_interface {
public:
    provider_base(const Json& js, const std::vector<Json>& etl, const Json& augmentation);
    // record idx of the window: params for every ETL element from one shared augmentation
    // (provider_base::provide, provider.cpp:109-119), then its pixels into the pinned arena
    void provide(int idx, const decoded_element* elems, decode_window& w, std::minstd_rand0& random) const;
    void draw(int idx, const decoded_element* elems, decode_window& w, std::minstd_rand0& random,
              light_split* ls = nullptr) const;
    // draw() for every record of a window with its own engine (deterministic mode), on the pool:
    // the same params as the in-order loop (the lighting cache hand-off is fixed up afterwards)
    void draw_window(int n, const decoded_element* records, decode_window& w, std::vector<std::minstd_rand0>& engines,
                     thread_pool& pool) const;
    void stage(int idx, const decoded_element* elems, decode_window& w) const;
    // aeon's vestigial post_process hook, used as the per-window GPU flush: outputs[k] receives
    // n items of provider k (device pointers if on_device, else host memory)
    void post_process(aeon_hip_ctx* ctx, decode_window& w, const uint8_t* dev_arena, void* const* outputs,
                      void* stream) const;
    const std::vector<std::unique_ptr<etl_provider>>& providers() const { return m_providers; }

private:
    std::vector<std::unique_ptr<etl_provider>> m_providers;
};

struct provider_factory {
    static std::shared_ptr<provider_base> create(const Json& config);
};

// thread_pool (src/thread_pool.hpp:82-175): persistent workers, worker i pinned to CPU
// affinity_map[i] (pthread_setaffinity_np, thread_pool.hpp:133-138); run(n, fn) hands out task ids
// from one atomic counter; the first exception is kept and rethrown after the barrier.
class thread_pool {
public:
    // one worker per entry of affinity_map (at least one; an empty map = one unpinned worker)
    explicit thread_pool(std::vector<int> affinity_map);
    ~thread_pool();
    void run(int n, const std::function<void(int)>& fn);
    // fn(task, worker): worker in [0, size()) identifies the calling pool thread
    void run_indexed(int n, const std::function<void(int, int)>& fn);
    int  size() const { return m_nthreads; }
    const std::vector<int>& affinity_map() const { return m_map; }
    // what worker i's own sched_getaffinity returned after it pinned itself (blocks until every
    // worker has started); a CPU outside the process's cpuset cannot be pinned to, and that worker
    // keeps the process mask -- aeon ignores pthread_setaffinity_np's result the same way
    std::vector<std::vector<int>> worker_cpus();

private:
    void                                 worker(int index);
    std::vector<int>                     m_map;
    std::vector<std::vector<int>>        m_worker_cpus;
    int                                  m_started = 0, m_nthreads = 0;
    std::vector<std::thread>             m_threads;
    std::mutex                           m_mu;
    std::condition_variable              m_cv, m_done_cv;
    const std::function<void(int, int)>* m_fn = nullptr;
    int                            m_n = 0;
    std::atomic<int>               m_done{0}; // tasks of the current run completed
    long                           m_generation = 0;
    std::atomic<uint64_t>          m_state{0}; // (generation << 32) | next task: a task is taken only in its own run
    std::exception_ptr             m_error;
    bool                           m_stop = false;
};

// batch_decoder: decode windows of records on the pool, flush each window to the GPU.
// Two window slots (async_manager's two containers, src/async_manager.hpp:203-204), each with its
// own pinned staging, device buffers, stream and completion event: submit() stages window k+1 and
// enqueues its copies and kernels while window k's are still running; wait() completes the oldest.
class batch_decoder {
public:
    batch_decoder(const Json& config, int device);
    ~batch_decoder();
    // n records x input_count elements (row-major); outputs[k] per provider buffer.  Synchronous,
    // on `stream` (batch_decoder::filler, src/batch_decoder.cpp:73-99).
    void decode(int n, const decoded_element* records, void* const* outputs, bool outputs_on_device,
                void* stream);
    // Asynchronous window on the decoder's own streams: returns once the records' bytes are
    // consumed (drawn, staged, entropy-decoded); outputs are complete after the matching wait().
    void submit(int n, const decoded_element* records, void* const* outputs, bool outputs_on_device);
    void wait(); // oldest submitted window
    // the draw phase of one window alone (host only): params[i] = record i's (first element's)
    // params; serial = the in-order loop instead of draw_window
    void draw_params(int n, const decoded_element* records, aeon_aug_params* params, bool serial);
    int  outstanding() const { return (int)m_queue.size(); }
    provider_base& provider() { return *m_provider; }
    thread_pool&   pool() { return *m_pool; }
    int            batch_size() const { return m_batch_size; }

private:
    struct window_slot {
        hipStream_t           stream  = nullptr;
        hipEvent_t            done    = nullptr;
        bool                  pending = false;
        uint8_t*              pinned = nullptr;
        size_t                pinned_cap = 0;
        uint8_t*              dev_src = nullptr;
        size_t                dev_src_cap = 0;
        std::vector<uint8_t*> dev_out, dev_tmp;
        std::vector<size_t>   dev_out_cap, dev_tmp_cap;
    };
    void enqueue(window_slot& ws, int n, const decoded_element* records, void* const* outputs, bool on_device,
                 hipStream_t stream);
    void                           grow_slot_engines(int n);
    std::shared_ptr<provider_base> m_provider;
    int                            m_batch_size = 1;
    bool                           m_deterministic = false;
    std::vector<std::minstd_rand0> m_random; // one engine per decode slot (batch_decoder.cpp:47-54)
    std::minstd_rand0              m_seed_gen; // seeds m_random[i] (grow_slot_engines)
    std::minstd_rand0              m_local_random; // non-deterministic mode (util.cpp:266)
    std::unique_ptr<thread_pool>   m_pool;
    aeon_hip_ctx*                  m_ctx = nullptr;
    int                            m_device = 0;
    window_slot                    m_slots[2];
    int                            m_next = 0;
    std::vector<int>               m_queue; // submitted, not yet waited (slot indices, oldest first)
    // batch_major=false (loader.hpp:63): outputs are produced batch-major into dev_tmp and
    // transposed per batch into the caller's layout (batch_iterator.cpp:125-136)
    bool                           m_batch_major = true;
};

// manifest_file node slicing (generate_blocks, src/manifest_file.cpp:278-295)
std::vector<int64_t> manifest_node_slice(int64_t record_count, int batch_size, int node_id, int node_count);

// nervana::parse_cpu_list (src/util.cpp:283-330): "0-4,30,10" -> sorted, de-duplicated CPU ids;
// std::invalid_argument for an id >= hardware_concurrency
std::vector<int> parse_cpu_list(const std::string& cpu_list);
// nervana::get_thread_affinity_map (src/util.cpp:337-373): AEON_CPU_LIST over the config's cpu_list;
// else hc - min(2, hc/8) CPUs.  aeon's default is iota(0, ...); here it is the first CPUs of the
// process's own affinity mask (the same list on an unrestricted host; inside a container given 16
// of 256 CPUs, CPUs the workers can actually be pinned to), capped by OMP_NUM_THREADS.
std::vector<int> thread_affinity_map(const std::string& cpu_list);
int aeon_thread_count(const std::string& cpu_list); // thread_affinity_map(cpu_list).size()
// the decoder's pool runs its context's JPEG entropy decoding too (stage.cpp)
void ctx_share_pool(aeon_hip_ctx* ctx, thread_pool* pool);
// a map stretched or cut to n workers (decode_thread_count / AEON_HIP_JPEG_THREADS): worker i on map[i % size]
std::vector<int> affinity_for(const std::vector<int>& map, int n);

} // namespace aeon_hip
