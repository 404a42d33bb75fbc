// host.cpp -- provider plugin surface + decode stage of the HIP image path (see host.hpp).
#include "host.hpp"

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <numeric>
#include <set>
#include <sstream>
#include <stdexcept>

namespace aeon_hip {

namespace {

[[noreturn]] void invalid(const std::string& m) { throw std::invalid_argument(m); }

void hip_check(hipError_t e, const char* what)
{
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void check(int rc)
{
    if (rc != 0) {
        int code = rc;
        std::string msg = aeon_hip_last_error();
        if (code == AEON_HIP_EINVAL) throw std::invalid_argument(msg);
        throw std::runtime_error(msg);
    }
}

size_t levenshtein(const std::string& a, const std::string& b)
{
    std::vector<size_t> v0(b.size() + 1), v1(b.size() + 1);
    std::iota(v0.begin(), v0.end(), 0);
    for (size_t i = 0; i < a.size(); i++) {
        v1[0] = i + 1;
        for (size_t j = 0; j < b.size(); j++)
            v1[j + 1] = std::min({v1[j] + 1, v0[j + 1] + 1, v0[j] + (a[i] == b[j] ? 0 : 1)});
        std::swap(v0, v1);
    }
    return v0[b.size()];
}

// interface.cpp verify_config: unknown keys are an error, with the closest known key suggested
void verify_config(const std::string& where, const std::set<std::string>& known, const Json& js)
{
    for (const auto& kv : js.object()) {
        if (known.count(kv.first)) continue;
        std::string best;
        size_t      best_d = (size_t)-1;
        for (const auto& k : known) {
            size_t d = levenshtein(kv.first, k);
            if (d < best_d) best_d = d, best = k;
        }
        invalid("config element {" + kv.first + "} is not understood in " + where +
                (best.empty() ? std::string() : ", did you mean {" + best + "}?"));
    }
}

template <typename T>
void get_num(const Json& js, const char* key, T& v)
{
    if (js.has(key)) v = (T)js.at(key).number();
}
void get_bool(const Json& js, const char* key, bool& v)
{
    if (js.has(key)) v = js.at(key).boolean();
}
void get_str(const Json& js, const char* key, std::string& v)
{
    if (js.has(key)) v = js.at(key).str();
}

Json without_type(const Json& j, std::string& type)
{
    if (!j.has("type")) invalid("missing required 'type' element in etl object");
    type = j.at("type").str();
    return j;
}

} // namespace

// ---- typemap -------------------------------------------------------------------------------
output_type::output_type(const std::string& n) : name(n)
{
    // typemap.hpp:43-52 (name -> cv type): the loader's convertTo target
    static const std::map<std::string, std::pair<size_t, int>> all{
        {"int8_t", {1, AEON_DTYPE_S8}},    {"uint8_t", {1, AEON_DTYPE_U8}},  {"int16_t", {2, AEON_DTYPE_S16}},
        {"uint16_t", {2, AEON_DTYPE_U16}}, {"int32_t", {4, AEON_DTYPE_S32}}, {"uint32_t", {4, AEON_DTYPE_S32}},
        {"float", {4, AEON_DTYPE_F32}},    {"double", {8, AEON_DTYPE_F64}},  {"char", {1, AEON_DTYPE_S8}}};
    auto it = all.find(n);
    if (it == all.end()) throw std::runtime_error("Unable to map output type " + n);
    size  = it->second.first;
    dtype = it->second.second;
}

bool output_type::is_valid_type(const std::string& n)
{
    try {
        output_type t(n);
        return true;
    } catch (...) {
        return false;
    }
}

size_t shape_type::byte_size() const
{
    size_t n = otype.size;
    for (size_t d : shape) n *= d;
    return n;
}

// ---- image::config (etl_image.cpp:25-65) ------------------------------------------------------
image_config::image_config(const Json& js)
{
    if (js.is_null()) throw std::runtime_error("missing image config in json config");
    if (!js.has("height")) invalid("Required Argument: 'height' not set");
    if (!js.has("width")) invalid("Required Argument: 'width' not set");
    get_num(js, "height", height);
    get_num(js, "width", width);
    get_str(js, "name", name);
    get_bool(js, "bgr_to_rgb", bgr_to_rgb);
    get_bool(js, "channel_major", channel_major);
    get_num(js, "channels", channels);
    if (!(channels == 1 || channels == 3)) invalid("value for 'channels' out of range");
    get_str(js, "output_type", output_type_name);
    if (!output_type::is_valid_type(output_type_name)) invalid("value for 'output_type' out of range");
    verify_config("image", {"type", "height", "width", "name", "bgr_to_rgb", "channel_major", "channels",
                            "output_type"},
                  js);
    if (js.at("height").number() <= 0) invalid("invalid height");
    if (js.at("width").number() <= 0) invalid("invalid width");
    if (bgr_to_rgb && channels != 3)
        invalid("invalid config: bgr_to_rgb can be 'true' only for channels set to '3'");
    shape.otype = output_type(output_type_name);
    if (channel_major) {
        shape.shape = {channels, height, width};
        shape.names = {"channels", "height", "width"};
    } else {
        shape.shape = {height, width, channels};
        shape.names = {"height", "width", "channels"};
    }
}

// ---- providers --------------------------------------------------------------------------------
const shape_type& provider_interface::get_output_shape(const std::string& name) const
{
    for (const auto& p : m_output_shapes)
        if (p.first == name) return p.second;
    throw std::runtime_error("key '" + name + "' not found");
}

const std::vector<std::string>& provider_interface::get_buffer_names()
{
    if (m_buffer_names.empty())
        for (const auto& p : m_output_shapes) m_buffer_names.push_back(p.first);
    return m_buffer_names;
}

namespace {

std::string create_name(const std::string& name, const std::string& base)
{
    return name.empty() ? base : name + "." + base;
}

// provider::image (provider.cpp:145-184): make_params when the record has none yet,
// transform_single_image + image::loader::load on the GPU at post_process time.
class image_provider : public etl_provider {
public:
    image_provider(const Json& js, const Json& aug)
        : m_cfg(js), m_factory(aug), m_name(create_name(m_cfg.name, "image"))
    {
        // image::loader ctor (etl_image.cpp:204-244)
        const auto& mean = m_factory.mean;
        const auto& std_ = m_factory.stddev;
        if (!mean.empty() || !std_.empty()) {
            if (!(m_cfg.output_type_name == "float" || m_cfg.output_type_name == "double"))
                invalid("Standardization (mean, stddev) is supported only for float or double 'output_type'.");
            if (mean.size() != m_cfg.channels || std_.size() != m_cfg.channels)
                invalid("Size of 'mean' and 'stddev' must be equal to number of channels or empty.");
        }
    }
    void provide(int, const decoded_element& in, augmentation& aug, std::minstd_rand0& random,
                 aeon_aug_params& params, light_split* ls) const override
    {
        if (!aug.has) {
            if (ls)
                m_factory.make_params_split(random, in.width, in.height, (int)m_cfg.width, (int)m_cfg.height,
                                            ls->entry_avail, &aug.image, &ls->exit_saved);
            else
                m_factory.make_params(random, in.width, in.height, (int)m_cfg.width, (int)m_cfg.height, &aug.image);
            aug.has = true;
        }
        params = aug.image;
    }
    const param_factory& factory() const override { return m_factory; }
    bool               is_mask() const override { return false; }
    const shape_type&  shape() const override { return m_cfg.shape; }
    const std::string& buffer_name() const override { return m_name; }
    aeon_out_desc      out_desc() const override
    {
        aeon_out_desc o{};
        o.dtype         = m_cfg.shape.otype.dtype;
        o.channels      = (int)m_cfg.channels;
        o.channel_major = m_cfg.channel_major;
        o.bgr_to_rgb    = m_cfg.bgr_to_rgb;
        o.has_mean      = !m_factory.mean.empty();
        for (size_t i = 0; i < m_factory.mean.size() && i < 3; i++)
            o.mean[i] = m_factory.mean[i], o.stddev[i] = m_factory.stddev[i];
        o.item_stride = m_cfg.shape.byte_size();
        o.fixed_aspect_ratio = m_factory.fixed_aspect_ratio;
        o.canvas_w = (int)m_cfg.width, o.canvas_h = (int)m_cfg.height;
        return o;
    }

private:
    image_config  m_cfg;
    param_factory m_factory;
    std::string   m_name;
};

// provider::pixelmask (provider.cpp:353-393): shares the record's image params.
class pixelmask_provider : public etl_provider {
public:
    pixelmask_provider(const Json& js, const Json& aug)
        : m_cfg(js), m_factory(aug), m_name(create_name(m_cfg.name, "pixelmask"))
    {
    }
    void provide(int, const decoded_element& in, augmentation& aug, std::minstd_rand0& random,
                 aeon_aug_params& params, light_split* ls) const override
    {
        if (!aug.has) {
            if (ls)
                m_factory.make_params_split(random, in.width, in.height, (int)m_cfg.width, (int)m_cfg.height,
                                            ls->entry_avail, &aug.image, &ls->exit_saved);
            else
                m_factory.make_params(random, in.width, in.height, (int)m_cfg.width, (int)m_cfg.height, &aug.image);
            aug.has = true;
        }
        params = aug.image;
    }
    const param_factory& factory() const override { return m_factory; }
    bool               is_mask() const override { return true; }
    const shape_type&  shape() const override { return m_cfg.shape; }
    const std::string& buffer_name() const override { return m_name; }
    aeon_out_desc      out_desc() const override
    {
        aeon_out_desc o{};
        o.dtype         = m_cfg.shape.otype.dtype;
        o.channels      = (int)m_cfg.channels;
        o.channel_major = m_cfg.channel_major;
        o.item_stride   = m_cfg.shape.byte_size();
        o.fixed_aspect_ratio = m_factory.fixed_aspect_ratio;
        o.canvas_w = (int)m_cfg.width, o.canvas_h = (int)m_cfg.height;
        return o;
    }

private:
    image_config  m_cfg;
    param_factory m_factory;
    std::string   m_name;
};

} // namespace

provider_base::provider_base(const Json& js, const std::vector<Json>& etl, const Json& aug)
    : provider_interface(js, etl.size())
{
    for (const Json& j : etl) {
        std::string type;
        without_type(j, type);
        std::unique_ptr<etl_provider> p;
        if (type == "image") p.reset(new image_provider(j, aug));
        else if (type == "pixelmask") p.reset(new pixelmask_provider(j, aug));
        else if (type == "label" || type == "localization_rcnn" || type == "localization_ssd" ||
                 type == "boundingbox" || type == "blob" || type == "video" || type == "char_map" ||
                 type == "label_map")
            throw std::runtime_error("etl type '" + type + "' is outside the HIP image stage");
        else
            invalid("unsupported etl type '" + type + "'");
        m_output_shapes.emplace_back(p->buffer_name(), p->shape());
        m_providers.push_back(std::move(p));
    }
}

void provider_base::provide(int idx, const decoded_element* elems, decode_window& w,
                            std::minstd_rand0& random) const
{
    draw(idx, elems, w, random);
    stage(idx, elems, w);
}

void provider_base::draw(int idx, const decoded_element* elems, decode_window& w, std::minstd_rand0& random,
                         light_split* ls) const
{
    augmentation aug;
    for (size_t k = 0; k < m_providers.size(); k++) {
        const decoded_element& e = elems[k];
        if (!e.data || e.width <= 0 || e.height <= 0) {
            std::stringstream ss;
            ss << "received " << (m_providers[k]->is_mask() ? "pixelmask" : "encoded image")
               << " with size 0, at idx " << idx;
            throw std::runtime_error(ss.str());
        }
        m_providers[k]->provide(idx, e, aug, random, w.params[k][idx], ls);
    }
}

// aeon runs provide() -- make_params included -- on its pool threads (batch_decoder.cpp:62-71); with
// one engine per record the draws are independent but for the lighting normal_distribution's cache
// inside the shared factory (augment_image.hpp:153-185), which passes one value from a record to the
// next.  Record i makes exactly three normal draws, each toggling the cache, so whether it starts
// with a cached value is known before any record is drawn: every record draws on the pool with that
// entry state (make_params_split), and one in-order pass hands each cached value to the next record.
// The params equal the in-order loop's bit for bit (tests/test_host.py draw-window tests).
void provider_base::draw_window(int n, const decoded_element* records, decode_window& w,
                                std::vector<std::minstd_rand0>& engines, thread_pool& pool) const
{
    const size_t ne = m_providers.size();
    const param_factory& F = m_providers[0]->factory(); // the first element draws (aug.has after it)
    const bool               lit = F.lighting_on();
    std::vector<light_split> ls(lit ? n : 0);
    const bool               a0 = F.light_avail();
    for (int i = 0; i < (int)ls.size(); i++) ls[i].entry_avail = a0 != ((i & 1) != 0);
    // tasks of 32 consecutive records, each engine drawn from a local copy: eight engines share a
    // cache line, and threads drawing neighbouring records through them made the pool slower than
    // one thread (C3 window of 1024: 399 vs 374 us)
    // The engines advance in a scratch copy committed (with the lighting state) only once every
    // record drew: a record that throws (an element of size 0) leaves the decoder as it was.
    constexpr int kChunk = 32;
    std::vector<std::minstd_rand0> next(engines.begin(), engines.begin() + n);
    pool.run((n + kChunk - 1) / kChunk, [&](int t) {
        for (int i = t * kChunk; i < std::min(n, (t + 1) * kChunk); i++)
            draw(i, records + (size_t)i * ne, w, next[i], lit ? &ls[i] : nullptr);
    });
    std::copy(next.begin(), next.end(), engines.begin());
    if (!lit) return;
    float cached = F.light_saved();
    for (int i = 0; i < n; i++) {
        if (ls[i].entry_avail)
            for (size_t k = 0; k < ne; k++) w.params[k][i].lighting[0] = cached;
        else
            cached = ls[i].exit_saved;
    }
    F.set_light_state(!ls[n - 1].entry_avail, cached);
}

void provider_base::stage(int idx, const decoded_element* elems, decode_window& w) const
{
    for (size_t k = 0; k < m_providers.size(); k++) {
        const decoded_element& e = elems[k];
        if (e.encoded) continue; // decoded on the device, straight into the source arena
        const size_t row = (size_t)e.width * e.channels * e.elem_bytes;
        uint8_t*     dst = w.arena + w.offset[k][idx];
        if (e.png_mode >= 0) { // extract on this pool thread, straight into the pinned arena
            check(aeon_decode_png(e.data, e.size, e.png_mode, dst, row, nullptr));
        } else if ((size_t)e.stride == row) {
            std::memcpy(dst, e.data, row * e.height);
        } else {
            for (int y = 0; y < e.height; y++) std::memcpy(dst + y * row, e.data + (size_t)y * e.stride, row);
        }
    }
}

void provider_base::post_process(aeon_hip_ctx* ctx, decode_window& w, const uint8_t* dev_arena,
                                 void* const* outputs, void* stream) const
{
    // image + pixelmask with the same params per record (provider.cpp:365-393): one pair call, whose
    // masks run inside the image launch
    if (m_providers.size() == 2 && !m_providers[0]->is_mask() && m_providers[1]->is_mask() && w.n > 0 &&
        std::memcmp(w.params[0].data(), w.params[1].data(), (size_t)w.n * sizeof(aeon_aug_params)) == 0) {
        aeon_out_desc io = m_providers[0]->out_desc(), mo = m_providers[1]->out_desc();
        check(aeon_hip_augment_pair_batch(ctx, w.n, w.descs[0].data(), dev_arena, w.descs[1].data(), dev_arena,
                                          w.params[0].data(), &io, outputs[0], &mo, outputs[1], stream));
        return;
    }
    for (size_t k = 0; k < m_providers.size(); k++) {
        const etl_provider& p = *m_providers[k];
        aeon_out_desc       o = p.out_desc();
        if (p.is_mask())
            check(aeon_hip_mask_batch(ctx, w.n, w.descs[k].data(), dev_arena, w.params[k].data(), &o,
                                      outputs[k], stream));
        else
            check(aeon_hip_augment_batch(ctx, w.n, w.descs[k].data(), dev_arena, w.params[k].data(), &o,
                                         outputs[k], stream));
    }
}

std::shared_ptr<provider_base> provider_factory::create(const Json& config)
{
    if (!config.has("etl")) invalid("required argument 'etl' not set");
    std::vector<Json> etl = config.at("etl").array();
    Json              aug;
    if (config.has("augmentation")) {
        const auto& a = config.at("augmentation").array();
        for (const Json& j : a)
            if (!j.has("type")) invalid("augmentation missing 'type'");
        if (!a.empty()) aug = a[0]; // provider_factory.cpp:39-43: only the first is used
    }
    return std::make_shared<provider_base>(config, etl, aug);
}

// ---- thread_pool ----------------------------------------------------------------------------------
thread_pool::thread_pool(std::vector<int> affinity_map) : m_map(std::move(affinity_map))
{
    // the worker count is fixed before any worker starts: a worker must not read m_threads while this
    // constructor is still growing it (ThreadSanitizer, tests/sanitize/host_driver.cpp)
    m_nthreads = std::max<int>(1, (int)m_map.size());
    m_worker_cpus.resize(m_nthreads);
    m_threads.reserve(m_nthreads);
    for (int i = 0; i < m_nthreads; i++) m_threads.emplace_back([this, i] { worker(i); });
}

thread_pool::~thread_pool()
{
    {
        std::lock_guard<std::mutex> l(m_mu);
        m_stop = true;
    }
    m_cv.notify_all();
    for (auto& t : m_threads) t.join();
}

std::vector<std::vector<int>> thread_pool::worker_cpus()
{
    std::unique_lock<std::mutex> l(m_mu);
    m_done_cv.wait(l, [&] { return m_started == m_nthreads; });
    return m_worker_cpus;
}

void thread_pool::worker(int index)
{
    // thread_pool.hpp:133-138: pin to thread_affinity_map[index] (the result is not checked there
    // either: a CPU outside the cpuset leaves the thread on the process mask)
    if (index < (int)m_map.size()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(m_map[index], &set);
        (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    {
        std::vector<int> cpus;
        cpu_set_t        got;
        if (sched_getaffinity(0, sizeof(got), &got) == 0)
            for (int c = 0; c < CPU_SETSIZE; c++)
                if (CPU_ISSET(c, &got)) cpus.push_back(c);
        std::lock_guard<std::mutex> l(m_mu);
        m_worker_cpus[index] = std::move(cpus);
        if (++m_started == m_nthreads) m_done_cv.notify_all();
    }
    long seen = 0;
    for (;;) {
        const std::function<void(int, int)>* fn;
        int                            n;
        {
            std::unique_lock<std::mutex> l(m_mu);
            m_cv.wait(l, [&] { return m_stop || m_generation != seen; });
            if (m_stop) return;
            seen = m_generation;
            fn   = m_fn;
            n    = m_n;
        }
        // dynamic task distribution (thread_pool.hpp:155-162), the task counter tagged with the run's
        // generation: a worker that wakes after its run completed (the caller has returned, fn is
        // gone) takes nothing, whatever run the counter belongs to by then
        uint64_t st = m_state.load();
        for (;;) {
            if ((uint32_t)(st >> 32) != (uint32_t)seen || (int)(uint32_t)st >= n) break;
            if (!m_state.compare_exchange_weak(st, st + 1)) continue;
            try {
                (*fn)((int)(uint32_t)st, index);
            } catch (...) {
                std::lock_guard<std::mutex> l(m_mu);
                if (!m_error) m_error = std::current_exception();
            }
            if (m_done.fetch_add(1) + 1 == n) {
                std::lock_guard<std::mutex> l(m_mu);
                m_done_cv.notify_all();
            }
            st = m_state.load();
        }
    }
}

void thread_pool::run(int n, const std::function<void(int)>& fn)
{
    run_indexed(n, [&](int i, int) { fn(i); });
}

void thread_pool::run_indexed(int n, const std::function<void(int, int)>& fn)
{
    // aeon's run() waits for every worker to check in (thread_pool.hpp:103-116); this one waits for the
    // n tasks: a pinned worker whose CPU another process holds no longer stalls the run until it is
    // scheduled (milliseconds on a shared host) when the others have done its share
    {
        std::lock_guard<std::mutex> l(m_mu);
        m_fn    = &fn;
        m_n     = n;
        m_error = nullptr;
        m_done  = 0;
        m_generation++;
        m_state = (uint64_t)(uint32_t)m_generation << 32;
    }
    m_cv.notify_all();
    std::unique_lock<std::mutex> l(m_mu);
    m_done_cv.wait(l, [&] { return m_done.load() >= n; });
    if (m_error) std::rethrow_exception(m_error); // thread_pool.hpp:113-115
}

// ---- batch_decoder -------------------------------------------------------------------------------
std::vector<int> parse_cpu_list(const std::string& cpu_list)
{
    std::vector<int>  cpus;
    std::stringstream ss(cpu_list);
    std::string       tok;
    try {
        while (std::getline(ss, tok, ',')) {
            if (tok.empty()) continue;
            const auto dash = tok.find('-');
            if (dash == std::string::npos) {
                cpus.push_back(std::stoi(tok));
            } else {
                const int from = std::stoi(tok.substr(0, dash)), to = std::stoi(tok.substr(dash + 1));
                for (int i = from; i <= to; i++) cpus.push_back(i);
            }
        }
    } catch (const std::exception&) {
        invalid("Failed to parse cpu list '" + cpu_list + "'");
    }
    std::sort(cpus.begin(), cpus.end());
    cpus.erase(std::unique(cpus.begin(), cpus.end()), cpus.end());
    const int hc = (int)std::thread::hardware_concurrency();
    if (!cpus.empty() && (cpus.front() < 0 || cpus.back() >= hc))
        invalid("One or more indexes computed from cpu list '" + cpu_list +
                "' exceed number of logical cores. Use values in range [0, " + std::to_string(hc - 1) + "].");
    return cpus;
}

std::vector<int> thread_affinity_map(const std::string& cpu_list)
{
    // util.cpp:337-373: the environment has precedence over the config
    std::string list = cpu_list;
    if (const char* e = std::getenv("AEON_CPU_LIST"))
        if (*e) list = e;
    std::vector<int> map = list.empty() ? std::vector<int>() : parse_cpu_list(list);
    if (!map.empty()) return map;
    // hc - min(2, hc/8) over the CPUs this process may run on (its affinity mask: the GPU box gives
    // each job 16 of its 256 CPUs, and workers pinned outside it would stay unpinned), further
    // capped by OMP_NUM_THREADS when the launcher sets it
    std::vector<int> allowed;
    cpu_set_t        set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0)
        for (int c = 0; c < CPU_SETSIZE; c++)
            if (CPU_ISSET(c, &set)) allowed.push_back(c);
    if (allowed.empty()) {
        allowed.resize(std::max(1u, std::thread::hardware_concurrency()));
        std::iota(allowed.begin(), allowed.end(), 0);
    }
    int hc = (int)allowed.size();
    if (const char* e = std::getenv("OMP_NUM_THREADS"))
        if (std::atoi(e) > 0) hc = std::min(hc, std::atoi(e));
    allowed.resize(std::max(1, hc - std::min(2, hc / 8)));
    return allowed;
}

int aeon_thread_count(const std::string& cpu_list) { return (int)thread_affinity_map(cpu_list).size(); }

std::vector<int> affinity_for(const std::vector<int>& map, int n)
{
    std::vector<int> out(std::max(1, n));
    for (size_t i = 0; i < out.size(); i++) out[i] = map.empty() ? -1 : map[i % map.size()];
    if (map.empty()) out.clear();
    return out;
}

batch_decoder::batch_decoder(const Json& config, int device) : m_device(device)
{
    verify_config("loader", {"manifest_filename", "manifest_root", "batch_size", "cache_directory",
                             "block_size", "batch_major", "subset_fraction", "shuffle_enable",
                             "shuffle_manifest", "cpu_list", "pinned", "random_seed", "iteration_mode",
                             "iteration_mode_count", "etl", "augmentation", "node_id", "node_count",
                             "ssd_config", "decode_thread_count"},
                  config);
    if (!config.has("batch_size")) invalid("Required Argument: 'batch_size' not set");
    get_num(config, "batch_size", m_batch_size);
    if (m_batch_size <= 0) invalid("batch_size must be > 0");
    uint32_t seed = 0, node_id = 0, node_count = 0;
    get_num(config, "random_seed", seed);
    get_num(config, "node_id", node_id);
    get_num(config, "node_count", node_count);
    if (node_count > 1) {
        if (node_id >= node_count) throw std::runtime_error("node_id can't be greater than node_count");
        if (seed == 0) seed = 1; // loader.cpp:109-113
    }
    get_bool(config, "batch_major", m_batch_major);
    std::string cpu_list;
    get_str(config, "cpu_list", cpu_list);
    std::vector<int> map = thread_affinity_map(cpu_list); // loader.cpp:159-171
    if (config.has("decode_thread_count")) { // (this stage's own knob: the map cycled or cut to it)
        int threads = 0;
        get_num(config, "decode_thread_count", threads);
        if (threads <= 0) invalid("decode_thread_count must be > 0");
        map = affinity_for(map, threads);
    }
    m_provider = provider_factory::create(config);
    m_pool.reset(new thread_pool(map));
    m_local_random.seed(std::random_device{}());
    // decoder seed = random_seed + node_id (loader.cpp:174); deterministic when non-zero
    const uint32_t dseed = seed ? seed + node_id : 0;
    m_deterministic      = dseed != 0;
    if (m_deterministic) m_seed_gen.seed(dseed); // slot engines: see slot_engines()
    // the HIP context is created on the first window (configs validate without a GPU)
}

batch_decoder::~batch_decoder()
{
    if (!m_ctx) return; // no window ran: nothing was allocated on the device
    (void)hipSetDevice(m_device);
    for (auto& ws : m_slots)
        if (ws.pending) (void)hipEventSynchronize(ws.done);
    aeon_hip_ctx_destroy(m_ctx);
    for (auto& ws : m_slots) {
        if (ws.done) (void)hipEventDestroy(ws.done);
        if (ws.stream) (void)hipStreamDestroy(ws.stream);
        if (ws.pinned) (void)hipHostFree(ws.pinned);
        if (ws.dev_src) (void)hipFree(ws.dev_src);
        for (auto* v : {&ws.dev_out, &ws.dev_tmp})
            for (auto* p : *v)
                if (p) (void)hipFree(p);
    }
}

// Deterministic mode: engine i of the decode window is seeded with the i-th output of
// minstd_rand0(random_seed + node_id) (batch_decoder.cpp:47-54).  aeon seeds decode_size engines
// up front; here the table grows with the largest window seen, continuing the same generator, so
// the first N engines are aeon's for any N.
void batch_decoder::grow_slot_engines(int n)
{
    while ((int)m_random.size() < n) {
        m_random.emplace_back();
        m_random.back().seed(m_seed_gen());
    }
}

namespace {
// Device address through which the kernels can store straight into host buffer p (pinned and
// mapped: hipHostMalloc / hipHostRegister), or null for pageable memory.  Such host outputs are
// written over PCIe by the augmentation (or transpose) kernels themselves -- zero-copy --, which
// measured 81.6 K against 54 K records/s host->host for C2 with a D2H copy behind the kernels
// (tools/e2e_probe.py): the kernels' store stream uses both PCIe directions' worth of requests in
// flight where the copy engine does not.  AEON_HIP_ZERO_COPY=0 keeps the device staging + D2H (the
// kernels then occupy the CUs only for their HBM-speed run; zero-copy holds them for the PCIe time).
void* zero_copy_view(void* p)
{
    static const bool on = [] {
        const char* e = std::getenv("AEON_HIP_ZERO_COPY");
        return !(e && std::atoi(e) == 0);
    }();
    if (!on || !p) return nullptr;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError(); // pageable memory: not an error
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return (uint8_t*)a.devicePointer + ((uint8_t*)p - (uint8_t*)a.hostPointer);
}

// A roctx range over one host phase of a decode window (rocprofv3 --marker-trace shows them
// next to the kernels: draw, stage, jpeg, augment, transpose, d2h).
struct phase_range {
    explicit phase_range(const char* name) { roctxRangePush(name); }
    ~phase_range() { roctxRangePop(); }
    phase_range(const phase_range&) = delete;
    phase_range& operator=(const phase_range&) = delete;
};

void grow_dev(uint8_t*& p, size_t& cap, size_t bytes)
{
    if (bytes <= cap) return;
    if (p) hip_check(hipFree(p), "hipFree");
    p = nullptr;
    hip_check(hipMalloc((void**)&p, bytes), "hipMalloc");
    cap = bytes;
}
} // namespace

// One decode window on `stream` using window slot ws (whose previous window has completed):
// batch_decoder::filler (batch_decoder.cpp:73-99) with the per-record body split into
//   host:   JPEG headers -> make_params (record order: aeon's deterministic draw order) ->
//           decoded pixels staged into pinned memory on the pool -> JPEG entropy decode
//   device: H2D of the staged pixels -> JPEG IDCT/colour into the source arena -> augmentation
//           kernels (post_process) -> [batch transpose] -> host outputs: stored there directly
//           when pinned (zero_copy_view), else staged on the device + one D2H
void batch_decoder::enqueue(window_slot& ws, int n, const decoded_element* in, void* const* outputs, bool on_device,
                            hipStream_t stream)
{
    const int ne = (int)m_provider->get_input_count();
    // image::extractor::extract of encoded elements: the frame header gives the decoded size; the
    // record is decoded with the provider's channel count (CV_LOAD_IMAGE_COLOR / GRAYSCALE)
    // (CV_LOAD_IMAGE_COLOR / GRAYSCALE for images, CV_LOAD_IMAGE_ANYDEPTH for pixel masks).  PNG
    // files are decoded on the host pool while staging (png_host.cpp), JPEG files on the device.
    std::vector<decoded_element> records(in, in + (size_t)n * ne);
    static const uint8_t kPngSig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    for (int i = 0; i < n; i++)
        for (int k = 0; k < ne; k++) {
            decoded_element& e = records[(size_t)i * ne + k];
            if (!e.encoded) continue;
            const bool mask = m_provider->providers()[k]->is_mask();
            const int  cn   = m_provider->providers()[k]->out_desc().channels;
            if (e.size >= 8 && std::memcmp(e.data, kPngSig, 8) == 0) {
                int depth = 0, ctype = 0;
                check(aeon_png_info(e.data, e.size, &e.width, &e.height, &depth, &ctype));
                e.encoded    = false;
                e.png_mode   = mask ? AEON_PNG_ANYDEPTH : (cn == 3 ? AEON_PNG_BGR8 : AEON_PNG_GRAY8);
                e.channels   = mask ? 1 : cn;
                e.elem_bytes = (mask && depth == 16 && ctype != 3) ? 2 : 1;
                e.stride     = e.width * e.channels * e.elem_bytes;
                continue;
            }
            if (mask)
                throw std::runtime_error("encoded pixel masks are decoded from PNG files only (JPEG masks: pass the "
                                         "decoded mask)");
            int comps = 0;
            check(aeon_jpeg_info(e.data, e.size, &e.width, &e.height, &comps));
            e.channels = cn;
            e.stride   = e.width * e.channels;
        }
    decode_window w;
    w.n = n;
    w.descs.assign(ne, std::vector<aeon_img_desc>(n));
    w.params.assign(ne, std::vector<aeon_aug_params>(n));
    w.offset.assign(ne, std::vector<size_t>(n));
    // source arena: decoded elements first (staged + one H2D), then the device-decoded JPEGs
    size_t staged = 0, total = 0;
    for (int pass = 0; pass < 2; pass++)
        for (int i = 0; i < n; i++)
            for (int k = 0; k < ne; k++) {
                const decoded_element& e = records[(size_t)i * ne + k];
                if (e.encoded != (pass == 1)) continue;
                const size_t b = (size_t)std::max(e.width, 0) * std::max(e.height, 0) * std::max(e.channels, 0) *
                                 e.elem_bytes;
                w.offset[k][i] = total;
                w.descs[k][i]  = aeon_img_desc{total, e.width, e.height, e.width * e.channels * e.elem_bytes, e.channels,
                                              e.elem_bytes == 2 ? 2 : 0, 0};
                total += (b + 15) & ~(size_t)15;
                if (pass == 0) staged = total;
            }
    total = std::max<size_t>(total, 16);
    if (staged > ws.pinned_cap) {
        if (ws.pinned) hip_check(hipHostFree(ws.pinned), "hipHostFree");
        ws.pinned = nullptr;
        hip_check(hipHostMalloc((void**)&ws.pinned, staged, hipHostMallocDefault), "hipHostMalloc");
        ws.pinned_cap = staged;
    }
    grow_dev(ws.dev_src, ws.dev_src_cap, total);
    w.arena = ws.pinned;
    // batch_decoder::process: the slot engine of record i draws its params (deterministic mode
    // swaps the slot engine in and out, batch_decoder.cpp:62-71).  With slot engines the draws run
    // on the pool (draw_window: aeon's in-order params exactly); then the pool threads stage the
    // pixels into the pinned arena.
    {
        phase_range r("aeon.draw");
        if (m_deterministic) {
            m_provider->draw_window(n, records.data(), w, m_random, *m_pool);
        } else { // one engine for the window: in record order
            for (int i = 0; i < n; i++) m_provider->draw(i, records.data() + (size_t)i * ne, w, m_local_random);
        }
    }
    if (staged) {
        {
            phase_range r("aeon.stage");
            m_pool->run(n, [&](int i) { m_provider->stage(i, records.data() + (size_t)i * ne, w); });
        }
        phase_range r("aeon.h2d_enqueue");
        hip_check(hipMemcpyAsync(ws.dev_src, ws.pinned, staged, hipMemcpyHostToDevice, stream), "hipMemcpyAsync");
    }
    for (int k = 0; k < ne; k++) {
        phase_range r("aeon.jpeg");
        std::vector<const void*> files;
        std::vector<size_t>      sizes;
        std::vector<aeon_img_desc> descs;
        for (int i = 0; i < n; i++) {
            const decoded_element& e = records[(size_t)i * ne + k];
            if (!e.encoded) continue;
            files.push_back(e.data), sizes.push_back(e.size), descs.push_back(w.descs[k][i]);
        }
        if (!files.empty())
            check(aeon_hip_decode_jpeg_batch(m_ctx, (int)files.size(), files.data(), sizes.data(), descs.data(),
                                             ws.dev_src, stream));
    }
    std::vector<void*> outs(ne);
    std::vector<bool>  copy_out(ne, false); // staged on the device, then one D2H into outputs[k]
    ws.dev_out.resize(ne, nullptr), ws.dev_out_cap.resize(ne, 0);
    ws.dev_tmp.resize(ne, nullptr), ws.dev_tmp_cap.resize(ne, 0);
    for (int k = 0; k < ne; k++) {
        const size_t bytes = (size_t)n * m_provider->providers()[k]->shape().byte_size();
        if (on_device) outs[k] = outputs[k];
        else if (void* v = zero_copy_view(outputs[k])) outs[k] = v;
        else {
            grow_dev(ws.dev_out[k], ws.dev_out_cap[k], bytes);
            outs[k]     = ws.dev_out[k];
            copy_out[k] = true;
        }
    }
    phase_range launch("aeon.launch");
    if (m_batch_major) {
        m_provider->post_process(m_ctx, w, ws.dev_src, outs.data(), stream);
    } else {
        std::vector<void*> tmp(ne);
        for (int k = 0; k < ne; k++) {
            grow_dev(ws.dev_tmp[k], ws.dev_tmp_cap[k], (size_t)n * m_provider->providers()[k]->shape().byte_size());
            tmp[k] = ws.dev_tmp[k];
        }
        m_provider->post_process(m_ctx, w, ws.dev_src, tmp.data(), stream);
        for (int k = 0; k < ne; k++) {
            const shape_type& sh    = m_provider->providers()[k]->shape();
            const size_t      esize = sh.otype.size;
            const size_t      item  = sh.byte_size();
            for (int b = 0; b < n / m_batch_size; b++) {
                const size_t off = (size_t)b * m_batch_size * item;
                check(aeon_hip_transpose_batch(m_ctx, (uint8_t*)tmp[k] + off, (uint8_t*)outs[k] + off,
                                               m_batch_size, (int64_t)(item / esize), (int)esize, stream));
            }
        }
    }
    for (int k = 0; k < ne; k++)
        if (copy_out[k]) {
            phase_range d2h("aeon.d2h_enqueue");
            hip_check(hipMemcpyAsync(outputs[k], outs[k], (size_t)n * m_provider->providers()[k]->shape().byte_size(),
                                     hipMemcpyDeviceToHost, stream),
                      "hipMemcpyAsync");
        }
    if (!ws.done) hip_check(hipEventCreateWithFlags(&ws.done, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(ws.done, stream), "hipEventRecord");
    ws.pending = true;
}

void batch_decoder::draw_params(int n, const decoded_element* records, aeon_aug_params* params, bool serial)
{
    if (n <= 0) return;
    const int ne = (int)m_provider->get_input_count();
    if (m_deterministic) grow_slot_engines(n);
    decode_window w;
    w.n = n;
    w.params.assign(ne, std::vector<aeon_aug_params>(n));
    if (m_deterministic && !serial) {
        m_provider->draw_window(n, records, w, m_random, *m_pool);
    } else {
        for (int i = 0; i < n; i++)
            m_provider->draw(i, records + (size_t)i * ne, w, m_deterministic ? m_random[i] : m_local_random);
    }
    std::copy(w.params[0].begin(), w.params[0].end(), params);
}

void batch_decoder::decode(int n, const decoded_element* records, void* const* outputs, bool on_device, void* stream_)
{
    if (n <= 0) return;
    if (!m_batch_major && n % m_batch_size != 0) invalid("batch_major=false needs whole batches per decode window");
    while (!m_queue.empty()) wait(); // windows are completed in submission order
    if (m_deterministic) grow_slot_engines(n);
    if (!m_ctx) check(aeon_hip_ctx_create(m_device, &m_ctx)), ctx_share_pool(m_ctx, m_pool.get());
    hip_check(hipSetDevice(m_device), "hipSetDevice");
    window_slot& ws = m_slots[m_next];
    m_next ^= 1;
    if (ws.pending) hip_check(hipEventSynchronize(ws.done), "hipEventSynchronize");
    ws.pending = false;
    enqueue(ws, n, records, outputs, on_device, (hipStream_t)stream_);
    // the pinned arena and the window's params must outlive the copies: finish the window
    check(aeon_hip_synchronize(m_ctx, stream_));
    ws.pending = false;
}

void batch_decoder::submit(int n, const decoded_element* records, void* const* outputs, bool on_device)
{
    if (n <= 0) invalid("empty decode window");
    if (!m_batch_major && n % m_batch_size != 0) invalid("batch_major=false needs whole batches per decode window");
    if (m_queue.size() >= 2) invalid("two windows are in flight: wait() for the oldest before submitting another");
    if (m_deterministic) grow_slot_engines(n);
    if (!m_ctx) check(aeon_hip_ctx_create(m_device, &m_ctx)), ctx_share_pool(m_ctx, m_pool.get());
    hip_check(hipSetDevice(m_device), "hipSetDevice");
    const int    slot = m_next;
    window_slot& ws   = m_slots[slot];
    m_next ^= 1;
    if (!ws.stream) hip_check(hipStreamCreateWithFlags(&ws.stream, hipStreamNonBlocking), "hipStreamCreate");
    if (ws.pending) hip_check(hipEventSynchronize(ws.done), "hipEventSynchronize");
    ws.pending = false;
    enqueue(ws, n, records, outputs, on_device, ws.stream);
    m_queue.push_back(slot);
}

void batch_decoder::wait()
{
    if (m_queue.empty()) invalid("no decode window in flight");
    const int slot = m_queue.front();
    m_queue.erase(m_queue.begin());
    window_slot& ws = m_slots[slot];
    check(aeon_hip_synchronize(m_ctx, ws.stream));
    ws.pending = false;
}

// ---- manifest_file node slicing ------------------------------------------------------------------
std::vector<int64_t> manifest_node_slice(int64_t record_count, int batch_size, int node_id, int node_count)
{
    std::vector<int64_t> out;
    if (node_count <= 1) {
        out.resize(record_count);
        std::iota(out.begin(), out.end(), 0);
        return out;
    }
    if (node_id < 0 || node_id >= node_count) invalid("node_id can't be greater than node_count");
    if (batch_size <= 0) invalid("batch_size must be > 0");
    const int64_t count   = record_count / node_count;
    const int64_t batches = count / batch_size;
    out.resize(count);
    for (int64_t i = 0; i < batches * batch_size; i++) {
        const int64_t batch_num = i / batch_size, in_batch = i % batch_size;
        out[i] = batch_num * batch_size * node_count + (int64_t)batch_size * node_id + in_batch;
    }
    const int64_t tail_count = count - batches * batch_size;
    const int64_t tail_src   = batches * batch_size * node_count + tail_count * node_id;
    const int64_t tail_dst   = batches * batch_size;
    for (int64_t i = 0; i < tail_count; i++) out[i + tail_dst] = i + tail_src;
    return out;
}

} // namespace aeon_hip

// ---- C ABI of the host layer ---------------------------------------------------------------------
struct aeon_decoder {
    std::unique_ptr<aeon_hip::batch_decoder> d;
};

namespace {
thread_local std::string g_host_err;

template <typename F>
int host_guarded(F&& f)
{
    try {
        f();
        return 0;
    } catch (const std::invalid_argument& e) {
        g_host_err = e.what();
        return AEON_HIP_EINVAL;
    } catch (const std::exception& e) {
        g_host_err = e.what();
        return AEON_HIP_ERUNTIME;
    }
}
} // namespace

namespace {
std::vector<aeon_hip::decoded_element> to_elements(aeon_decoder* d, int n, const aeon_encoded_elem* elems)
{
    const int ne = (int)d->d->provider().get_input_count();
    std::vector<aeon_hip::decoded_element> recs((size_t)n * ne);
    for (size_t i = 0; i < recs.size(); i++) {
        const aeon_encoded_elem& e = elems[i];
        aeon_hip::decoded_element& r = recs[i];
        r.data = (const uint8_t*)e.data;
        if (e.width > 0) {
            r.width = e.width, r.height = e.height, r.channels = e.channels;
            r.stride = e.stride ? e.stride : e.width * e.channels;
        } else {
            if (!e.data || !e.size) throw std::runtime_error("received encoded image with size 0, at idx " +
                                                             std::to_string(i / ne));
            r.encoded = true, r.size = e.size;
        }
    }
    return recs;
}
} // namespace

extern "C" {

int aeon_decoder_create(const char* config_json, int device, aeon_decoder** out)
{
    return host_guarded([&] {
        if (!out || !config_json) throw std::invalid_argument("null argument");
        auto* d = new aeon_decoder();
        try {
            d->d.reset(new aeon_hip::batch_decoder(aeon_hip::Json::parse(config_json), device));
        } catch (...) {
            delete d;
            throw;
        }
        *out = d;
    });
}

int aeon_decoder_destroy(aeon_decoder* d)
{
    delete d;
    return 0;
}

int aeon_decoder_output_count(aeon_decoder* d, int* count)
{
    return host_guarded([&] {
        if (!d || !count) throw std::invalid_argument("null argument");
        *count = (int)d->d->provider().get_output_shapes().size();
    });
}

int aeon_decoder_output_info(aeon_decoder* d, int index, char* name, size_t name_cap, int64_t* shape,
                             int* ndim, size_t* item_bytes, int* dtype)
{
    return host_guarded([&] {
        if (!d) throw std::invalid_argument("null decoder");
        const auto& shapes = d->d->provider().get_output_shapes();
        if (index < 0 || index >= (int)shapes.size()) throw std::invalid_argument("output index out of range");
        const auto& s = shapes[index];
        if (name && name_cap) {
            std::strncpy(name, s.first.c_str(), name_cap - 1);
            name[name_cap - 1] = 0;
        }
        if (ndim) *ndim = (int)s.second.shape.size();
        if (shape)
            for (size_t i = 0; i < s.second.shape.size(); i++) shape[i] = (int64_t)s.second.shape[i];
        if (item_bytes) *item_bytes = s.second.byte_size();
        if (dtype) *dtype = s.second.otype.dtype;
    });
}

int aeon_decoder_decode(aeon_decoder* d, int n, const aeon_record_elem* elems, void* const* outputs,
                        int outputs_on_device, void* stream)
{
    return host_guarded([&] {
        if (!d || (n > 0 && (!elems || !outputs))) throw std::invalid_argument("null argument");
        const int ne = (int)d->d->provider().get_input_count();
        std::vector<aeon_hip::decoded_element> recs((size_t)n * ne);
        for (size_t i = 0; i < recs.size(); i++)
            recs[i] = aeon_hip::decoded_element{(const uint8_t*)elems[i].data, elems[i].width, elems[i].height,
                                                elems[i].channels,
                                                elems[i].stride ? elems[i].stride : elems[i].width * elems[i].channels};
        d->d->decode(n, recs.data(), outputs, outputs_on_device != 0, stream);
    });
}

int aeon_decoder_draw_params(aeon_decoder* d, int n, const aeon_record_elem* elems, aeon_aug_params* params,
                             int serial)
{
    return host_guarded([&] {
        if (!d || (n > 0 && (!elems || !params))) throw std::invalid_argument("null argument");
        const int ne = (int)d->d->provider().get_input_count();
        std::vector<aeon_hip::decoded_element> recs((size_t)n * ne);
        for (size_t i = 0; i < recs.size(); i++)
            recs[i] = aeon_hip::decoded_element{(const uint8_t*)elems[i].data, elems[i].width, elems[i].height,
                                                elems[i].channels,
                                                elems[i].stride ? elems[i].stride : elems[i].width * elems[i].channels};
        d->d->draw_params(n, recs.data(), params, serial != 0);
    });
}

int aeon_decoder_decode_encoded(aeon_decoder* d, int n, const aeon_encoded_elem* elems, void* const* outputs,
                                int outputs_on_device, void* stream)
{
    return host_guarded([&] {
        if (!d || (n > 0 && (!elems || !outputs))) throw std::invalid_argument("null argument");
        auto recs = to_elements(d, n, elems);
        d->d->decode(n, recs.data(), outputs, outputs_on_device != 0, stream);
    });
}

int aeon_decoder_submit(aeon_decoder* d, int n, const aeon_encoded_elem* elems, void* const* outputs,
                        int outputs_on_device)
{
    return host_guarded([&] {
        if (!d || n <= 0 || !elems || !outputs) throw std::invalid_argument("null argument");
        auto recs = to_elements(d, n, elems);
        d->d->submit(n, recs.data(), outputs, outputs_on_device != 0);
    });
}

int aeon_decoder_wait(aeon_decoder* d)
{
    return host_guarded([&] {
        if (!d) throw std::invalid_argument("null argument");
        d->d->wait();
    });
}

int aeon_manifest_node_slice(int64_t record_count, int batch_size, int node_id, int node_count,
                             int64_t* indices, int64_t* count)
{
    return host_guarded([&] {
        if (!count) throw std::invalid_argument("null count");
        auto v = aeon_hip::manifest_node_slice(record_count, batch_size, node_id, node_count);
        if (indices) std::copy(v.begin(), v.end(), indices);
        *count = (int64_t)v.size();
    });
}

int aeon_thread_affinity_map(const char* cpu_list, int* cpus, int cap, int* count)
{
    return host_guarded([&] {
        if (!count || (cap > 0 && !cpus)) throw std::invalid_argument("null argument");
        const auto map = aeon_hip::thread_affinity_map(cpu_list ? cpu_list : "");
        for (int i = 0; i < std::min(cap, (int)map.size()); i++) cpus[i] = map[i];
        *count = (int)map.size();
    });
}

int aeon_decoder_pool_cpus(aeon_decoder* d, int worker, int* map_cpu, int* cpus, int cap, int* count)
{
    return host_guarded([&] {
        if (!d || !count || (cap > 0 && !cpus)) throw std::invalid_argument("null argument");
        aeon_hip::thread_pool& p = d->d->pool();
        if (worker < 0 || worker >= p.size()) throw std::invalid_argument("worker out of range");
        const auto all = p.worker_cpus();
        const auto& w  = all[worker];
        if (map_cpu) *map_cpu = worker < (int)p.affinity_map().size() ? p.affinity_map()[worker] : -1;
        for (int i = 0; i < std::min(cap, (int)w.size()); i++) cpus[i] = w[i];
        *count = (int)w.size();
    });
}

int aeon_decoder_pool_size(aeon_decoder* d, int* workers)
{
    return host_guarded([&] {
        if (!d || !workers) throw std::invalid_argument("null argument");
        *workers = d->d->pool().size();
    });
}

const char* aeon_decoder_last_error(void) { return g_host_err.c_str(); }

} // extern "C"
