// aeon_path_cpp.cpp -- aeon's own decode stage with the HIP stager in place of provide()'s pixel work,
// call for call, in C++ against libaeon_hip.so (INTEGRATION.md edits 1-5; tests/test_integration.py checks
// the same sequence bit for bit through the Python binding).
//
//   loader (/root/reference/src/loader.cpp:158-176): thread_affinity_map -> pool size T, decode_size = the
//     smallest multiple of batch_size holding 8 records per thread, seed random_seed + node_id
//   batch_decoder::filler (/root/reference/src/batch_decoder.cpp:73-99): per window, the pool runs
//     process(i) for i < decode_size -- provide(i % batch, record i, outputs[i / batch]) = make_params
//     from slot engine i (deterministic mode, :47-54) + aeon_hip_stager_stage (provider::image's pixel
//     half, INTEGRATION edit 3) -- then post_process per batch buffer (edits 1-2): launch-only with the
//     consumer waiting (edit 4, "overlap"), or a flush (launch + wait)
//   batch_iterator_fbm::filler (/root/reference/src/batch_iterator.cpp:109-142): the consumer takes each
//     batch out of the decoded container after aeon_hip_stager_wait(NULL, buffer)
//   async_manager (/root/reference/src/async_manager.hpp:162-204): two containers alternate
//   buffer_fixed_size_elements::allocate (/root/reference/src/buffer_batch.cpp:150-186, edit 5): batch
//     buffers pageable (new char[]) or, "pinned": true, from aeon_hip_host_alloc -- which the kernels
//     store into directly (zero-copy)
//
// The pool is T workers pinned one per CPU of aeon's thread_affinity_map (aeon_thread_affinity_map);
// records are synthetic decoded HWC uint8 images (the bench's splitmix64 pattern) held in host memory,
// as imdecode leaves them.  Prints one JSON line: records/s over the timed windows.
//
// usage: aeon_path_cpp <C1|C2> <pageable|pinned> <overlap|flush> [windows] [warmup] [batch]
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/aeon_hip.h"

namespace {

[[noreturn]] void die(const char* what, int rc, const char* msg)
{
    std::fprintf(stderr, "aeon_path_cpp: %s failed (%d): %s\n", what, rc, msg ? msg : "");
    std::exit(1);
}
#define HIP_CALL(expr)                                                  \
    do {                                                                \
        const int rc_ = (expr);                                         \
        if (rc_ != 0) die(#expr, rc_, aeon_hip_last_error());            \
    } while (0)
#define STAGER_CALL(expr)                                                \
    do {                                                                \
        const int rc_ = (expr);                                         \
        if (rc_ != 0) die(#expr, rc_, aeon_hip_stager_last_error());     \
    } while (0)

// aeon's thread_pool (src/thread_pool.hpp:106-174) reduced to what filler uses: run(n) hands indices
// 0..n-1 to the pinned workers and returns when all are processed.
class Pool {
public:
    explicit Pool(const std::vector<int>& cpus)
    {
        for (size_t w = 0; w < cpus.size(); w++)
            m_threads.emplace_back([this, cpu = cpus[w]] {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(cpu, &set);
                pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
                loop();
            });
    }
    ~Pool()
    {
        {
            std::lock_guard<std::mutex> l(m_mu);
            m_stop = true;
        }
        m_cv.notify_all();
        for (auto& t : m_threads) t.join();
    }
    void run(int n, const std::function<void(int)>& fn)
    {
        {
            std::lock_guard<std::mutex> l(m_mu);
            m_fn = &fn, m_n = n, m_next = 0, m_done = 0, m_gen++;
        }
        m_cv.notify_all();
        std::unique_lock<std::mutex> l(m_mu);
        m_done_cv.wait(l, [&] { return m_done == m_n; });
        m_fn = nullptr;
    }
    int size() const { return (int)m_threads.size(); }

private:
    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> l(m_mu);
                m_cv.wait(l, [&] { return m_stop || m_gen != seen; });
                if (m_stop) return;
                seen = m_gen, fn = m_fn;
            }
            int did = 0;
            for (;;) {
                const int i = m_next.fetch_add(1);
                if (i >= m_n) break;
                (*fn)(i);
                did++;
            }
            std::lock_guard<std::mutex> l(m_mu);
            m_done += did;
            if (m_done == m_n) m_done_cv.notify_all();
        }
    }
    std::vector<std::thread>        m_threads;
    std::mutex                      m_mu;
    std::condition_variable         m_cv, m_done_cv;
    const std::function<void(int)>* m_fn = nullptr;
    std::atomic<int>                m_next{0};
    int                             m_n = 0, m_done = 0;
    uint64_t                        m_gen = 0;
    bool                            m_stop = false;
};

template <typename T>
class Queue { // the async_manager hand-off between the decode thread and the consumer
public:
    void put(T v)
    {
        {
            std::lock_guard<std::mutex> l(m_mu);
            m_q.push_back(v);
        }
        m_cv.notify_one();
    }
    T get()
    {
        std::unique_lock<std::mutex> l(m_mu);
        m_cv.wait(l, [&] { return !m_q.empty(); });
        T v = m_q.front();
        m_q.pop_front();
        return v;
    }

private:
    std::mutex              m_mu;
    std::condition_variable m_cv;
    std::deque<T>           m_q;
};

// bench.py / aeon_amd.synthetic_image: byte = splitmix64(seed ^ (img << 32) ^ idx) & 0xff
void synthetic_image(uint64_t index, int w, int h, int cn, uint8_t* dst)
{
    const uint64_t seed = 0x5EED;
    for (uint64_t i = 0; i < (uint64_t)w * h * cn; i++) {
        uint64_t z = (seed ^ (index << 32) ^ i) + 0x9E3779B97F4A7C15ull;
        z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        dst[i]     = (uint8_t)((z ^ (z >> 31)) & 0xff);
    }
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <C1|C2> <pageable|pinned> <overlap|flush> [windows] [warmup] [batch]\n", argv[0]);
        return 2;
    }
    const std::string cfg = argv[1];
    const bool pinned  = std::strcmp(argv[2], "pinned") == 0;
    const bool overlap = std::strcmp(argv[3], "overlap") == 0;
    const int  windows = argc > 4 ? std::atoi(argv[4]) : 16;
    const int  warmup  = argc > 5 ? std::atoi(argv[5]) : 3;
    const bool c1      = cfg == "C1";
    const int  batch   = argc > 6 ? std::atoi(argv[6]) : (c1 ? 32 : 256);
    const int  src_w = c1 ? 480 : 256, src_h = c1 ? 360 : 256;
    // the loader's pool and decode window (loader.cpp:158-166)
    std::vector<int> cpus(1024);
    int              ncpu = 0;
    HIP_CALL(aeon_thread_affinity_map(nullptr, cpus.data(), (int)cpus.size(), &ncpu));
    cpus.resize(ncpu);
    const int decode_size = batch * ((ncpu * 8 - 1) / batch + 1);
    const int nb          = decode_size / batch;

    aeon_hip_ctx* ctx = nullptr;
    HIP_CALL(aeon_hip_ctx_create(0, &ctx));
    const char* aug_json =
        c1 ? R"({"type": "image", "center": true, "scale": [0.875, 0.875], "resize_short_size": 256, "flip_enable": false,
                "mean": [0.485, 0.456, 0.406], "stddev": [0.229, 0.224, 0.225]})"
           : R"({"type": "image", "center": false, "scale": [0.5, 1.0], "flip_enable": true,
                "mean": [0.485, 0.456, 0.406], "stddev": [0.229, 0.224, 0.225]})";
    aeon_param_factory* factory = nullptr;
    HIP_CALL(aeon_param_factory_create(aug_json, &factory));
    aeon_out_desc out{};
    out.dtype = AEON_DTYPE_F32, out.channels = 3, out.channel_major = 1, out.bgr_to_rgb = 1, out.has_mean = 1;
    const double mean[3] = {0.485, 0.456, 0.406}, stddev[3] = {0.229, 0.224, 0.225};
    for (int c = 0; c < 3; c++) out.mean[c] = mean[c], out.stddev[c] = stddev[c];
    out.item_stride = 3ull * 224 * 224 * 4;
    aeon_hip_stager* st = nullptr;
    STAGER_CALL(aeon_hip_stager_create(ctx, AEON_STAGER_IMAGE, &out, batch, &st));

    // decoded records (imdecode's output, host memory) and the slot engines (seed random_seed + node_id)
    const size_t         rec_bytes = (size_t)src_w * src_h * 3;
    std::vector<uint8_t> recs((size_t)decode_size * rec_bytes);
    for (int i = 0; i < decode_size; i++) synthetic_image(i, src_w, src_h, 3, recs.data() + i * rec_bytes);
    std::vector<uint32_t> engines(decode_size);
    HIP_CALL(aeon_seed_slots(1, decode_size, engines.data()));

    // two containers of nb batch buffers (buffer_fixed_size_elements::allocate, edit 5)
    const size_t              bbytes = (size_t)batch * out.item_stride;
    std::vector<std::vector<uint8_t*>> cont(2, std::vector<uint8_t*>(nb));
    for (auto& c : cont)
        for (auto& b : c) {
            if (pinned) HIP_CALL(aeon_hip_host_alloc(bbytes, (void**)&b));
            else b = new uint8_t[bbytes];
            std::memset(b, 0, bbytes);
        }

    Pool                pool(cpus);
    Queue<int>          free_q, full_q;
    free_q.put(0), free_q.put(1);
    const int           total = warmup + windows;
    std::chrono::steady_clock::time_point t0;
    std::atomic<bool>   failed{false};
    std::string         first_error;
    std::mutex          err_mu;

    std::thread decoder([&] { // batch_decoder::filler
        for (int w = 0; w < total; w++) {
            const int c = free_q.get();
            if (w == warmup) t0 = std::chrono::steady_clock::now();
            pool.run(decode_size, [&](int i) { // process(i) -> provider::image::provide
                aeon_aug_params p{};
                int rc = aeon_make_params(factory, &engines[i], src_w, src_h, 224, 224, &p);
                if (rc == 0)
                    rc = aeon_hip_stager_stage(st, cont[c][i / batch], i % batch, recs.data() + (size_t)i * rec_bytes, src_w,
                                               src_h, src_w * 3, 3, 1, &p);
                if (rc != 0 && !failed.exchange(true)) {
                    std::lock_guard<std::mutex> l(err_mu);
                    first_error = aeon_hip_stager_last_error();
                }
            });
            if (failed) die("provide", -1, first_error.c_str());
            for (int b = 0; b < nb; b++) // post_process per batch (edits 1-3)
                STAGER_CALL(overlap ? aeon_hip_stager_launch(st, cont[c][b]) : aeon_hip_stager_flush(st, cont[c][b]));
            full_q.put(c);
        }
    });
    uint64_t sink = 0;
    for (int w = 0; w < total; w++) { // batch_iterator_fbm::filler
        const int c = full_q.get();
        for (int b = 0; b < nb; b++) {
            STAGER_CALL(aeon_hip_stager_wait(nullptr, cont[c][b])); // (edit 4; flush mode: returns at once)
            sink += cont[c][b][0];
        }
        free_q.put(c);
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    decoder.join();
    std::printf("{\"cfg\": \"%s\", \"buffers\": \"%s\", \"post_process\": \"%s\", \"value\": %.1f, \"unit\": \"images/s\", "
                "\"ms_per_window\": %.3f, \"batch\": %d, \"decode_size\": %d, \"pool_threads\": %d, \"windows\": %d, "
                "\"sink\": %llu}\n",
                cfg.c_str(), pinned ? "pinned" : "pageable", overlap ? "launch+consumer wait" : "flush",
                (double)decode_size * windows / dt, dt / windows * 1e3, batch, decode_size, ncpu, windows,
                (unsigned long long)(sink & 1));
    STAGER_CALL(aeon_hip_stager_destroy(st));
    for (auto& c : cont)
        for (auto& b : c) {
            if (pinned) HIP_CALL(aeon_hip_host_free(b));
            else delete[] b;
        }
    HIP_CALL(aeon_param_factory_destroy(factory));
    HIP_CALL(aeon_hip_ctx_destroy(ctx));
    return 0;
}
