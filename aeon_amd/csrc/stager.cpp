// stager.cpp -- the aeon-side drop-in's staging + window launch (aeon_hip_stager_*, include/aeon_hip.h).
//
// aeon runs provide(idx, record, out_buf) for every record of a decode window on its pool and then
// (the one-line change) post_process(out_buf) once per batch of the window
// (src/batch_decoder.cpp:62-99).  A stager is what provider::image / provider::pixelmask hold to make
// those calls the GPU path:
//   stage(batch_out, idx, pixels, params)  -- provide(): the decoded record's bytes into pinned memory
//                                            (lock-free bump allocation in pinned chunks; concurrent)
//   launch(batch_out)                      -- post_process(): the FIRST call after a window's stages
//                                            launches the whole window -- one H2D per pinned chunk, ONE
//                                            augment (or mask) launch over every staged record of every
//                                            batch, one D2H per batch buffer (or, for pinned batch
//                                            buffers, the kernels store into them directly) -- on the
//                                            window's own stream, and returns
//   wait(batch_out)                        -- the consumer (batch_iterator_fbm::filler) before it swaps
//                                            or copies the batch: blocks until that batch is complete
//   flush(batch_out)                       -- launch + wait (post_process that returns a finished batch)
// Two windows are kept, as aeon's async_manager keeps two containers (src/async_manager.hpp:162-204):
// while window k's copies and kernels run, window k+1 stages into the other one.
// The batch buffer's own address (out_buf[name]->get_item(0)) is the staging key: batches of one
// window never share it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/aeon_hip.h"

namespace {

thread_local std::string g_stager_err;

struct stager_error : std::runtime_error {
    int code;
    stager_error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

[[noreturn]] void fail(int code, const std::string& m) { throw stager_error(code, m); }

void hip_ok(hipError_t e, const char* what)
{
    if (e != hipSuccess) fail(AEON_HIP_ERUNTIME, std::string(what) + ": " + hipGetErrorString(e));
}

void abi_ok(int rc)
{
    if (rc != 0) fail(rc, aeon_hip_last_error());
}

// Device address of pinned, device-mapped host memory p (hipHostMalloc / hipHostRegister), or null.
void* mapped_view(void* p)
{
    static const bool on = [] {
        const char* e = std::getenv("AEON_HIP_ZERO_COPY");
        return !(e && std::atoi(e) == 0);
    }();
    if (!on || !p) return nullptr;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError(); // pageable memory
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return (uint8_t*)a.devicePointer + ((uint8_t*)p - (uint8_t*)a.hostPointer);
}

constexpr size_t kChunkBytes = 64u << 20; // pinned staging chunk (a window usually fits in one or two)

struct Chunk {
    uint8_t* host = nullptr;
    size_t   cap  = 0;
    size_t   used = 0; // bump offset (under the stager's mutex)
    size_t   base = 0; // its offset in the device arena of the launched window
};

// One batch buffer of the window: per idx, where its pixels are and its params.
struct Batch {
    void*                        out = nullptr; // the batch buffer (host, or device memory)
    std::vector<aeon_img_desc>   descs;         // offset = (chunk << 48) | offset in chunk until launch
    std::vector<aeon_aug_params> params;
    std::unique_ptr<std::atomic<uint8_t>[]> have;
    int        first = 0;     // its first record in the window's launch order
    int        n     = 0;     // records staged (idx 0..n-1)
    hipEvent_t done  = nullptr;
    bool       d2h   = false; // pageable batch: its wait copies it out of the window's device outputs
    bool       launched = false; // a flush / launch named this batch buffer
    bool       waited   = false; // a flush / wait returned (or is returning) its completion
};

// A decode window: its pinned staging, its batches, its own stream and device buffers, so that window
// k's copies and kernels run while window k+1 is staged (aeon's async_manager keeps two containers in
// flight, src/async_manager.hpp:162-204).
struct Window {
    enum State { IDLE, STAGING, LAUNCHED };
    State                               state = IDLE;
    uint64_t                            gen   = 0; // launch generation (a retire checks it)
    std::vector<Chunk>                  chunks;
    int                                 cur = 0; // chunk being filled
    std::vector<std::unique_ptr<Batch>> batches; // in first-stage order
    int                                 unwaited = 0;
    hipStream_t                         stream  = nullptr;
    hipEvent_t                          done    = nullptr;
    uint8_t*                            dev_src = nullptr;
    size_t                              dev_src_cap = 0;
    uint8_t*                            dev_out = nullptr;
    size_t                              dev_out_cap = 0;
    std::atomic<int>                    copying{0}; // waits copying a pageable batch out of dev_out
};

} // namespace

struct aeon_hip_stager {
    aeon_hip_ctx* ctx   = nullptr;
    int           kind  = AEON_STAGER_IMAGE;
    aeon_out_desc out{};
    int           batch = 0;
    int           device = 0;
    std::mutex    mu;
    Window        win[2];
    int           cur = 0; // the window stages go to
    uint64_t      gens = 0;
    std::vector<hipEvent_t> spare_events;
    std::atomic<int>        waiters{0}; // aeon_hip_stager_wait(NULL, ...) calls inside this stager (destroy waits)
};

namespace {

// Batch buffers of launched windows -> their stager, for aeon_hip_stager_wait(NULL, buffer) (the
// consumer, batch_iterator_fbm::filler, knows the buffers but not the providers).  Lock order: a
// stager's mu may be held when g_reg_mu is taken, never the reverse.
// An entry is (stager, window generation): a buffer address that appears in both windows keeps the
// newer window's entry, and retiring the older window erases only its own.
struct Pending {
    aeon_hip_stager* s;
    uint64_t         gen;
};
std::mutex                        g_reg_mu;
std::unordered_map<void*, Pending> g_pending;

template <typename F>
int stager_guarded(F&& f)
{
    try {
        f();
        return 0;
    } catch (const stager_error& e) {
        g_stager_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_stager_err = e.what();
        return AEON_HIP_ERUNTIME;
    }
}

void grow(uint8_t*& p, size_t& cap, size_t need)
{
    if (need <= cap) return;
    const size_t n = std::max(need, cap + cap / 2);
    if (p) hip_ok(hipFree(p), "hipFree");
    p = nullptr, cap = 0;
    hip_ok(hipMalloc((void**)&p, n), "hipMalloc");
    cap = n;
}

// Forget a completed (or dropped) window: batches gone, chunks empty (their memory is kept).  Caller
// holds s->mu.
void reset_window(aeon_hip_stager* s, Window& w)
{
    if (w.state == Window::LAUNCHED) {
        std::lock_guard<std::mutex> r(g_reg_mu);
        for (auto& b : w.batches) {
            auto it = g_pending.find(b->out);
            if (it != g_pending.end() && it->second.s == s && it->second.gen == w.gen) g_pending.erase(it);
        }
    }
    for (auto& b : w.batches)
        if (b->done) s->spare_events.push_back(b->done);
    w.batches.clear();
    for (Chunk& c : w.chunks) c.used = 0;
    w.cur      = 0;
    w.state    = Window::IDLE;
    w.unwaited = 0;
}

// The window stages go to, under s->mu: the current one unless it was launched, else the other one --
// which, if it is still in flight (its consumer never waited for it), is completed and dropped first.
Window& staging_window(aeon_hip_stager* s)
{
    if (s->win[s->cur].state != Window::LAUNCHED) return s->win[s->cur];
    s->cur    = 1 - s->cur;
    Window& w = s->win[s->cur];
    if (w.state == Window::LAUNCHED) {
        hip_ok(hipSetDevice(s->device), "hipSetDevice");
        hip_ok(hipEventSynchronize(w.done), "hipEventSynchronize");
        // its pageable batches nobody waited for: their D2H now, so they are complete when this returns
        for (auto& b : w.batches)
            if (b->d2h && !b->waited) {
                b->waited = true;
                hip_ok(hipMemcpy(b->out, w.dev_out + (size_t)b->first * s->out.item_stride, (size_t)b->n * s->out.item_stride,
                                 hipMemcpyDeviceToHost),
                       "hipMemcpy");
            }
        while (w.copying.load(std::memory_order_acquire) != 0) std::this_thread::yield();
        reset_window(s, w);
    }
    return w;
}

// Reserve `bytes` (16-aligned) of pinned staging: returns (chunk, offset).  Caller holds s->mu.
std::pair<int, size_t> reserve(Window& w, size_t bytes)
{
    bytes = (bytes + 15) & ~(size_t)15;
    for (;; w.cur++) {
        if (w.cur == (int)w.chunks.size()) {
            Chunk c;
            c.cap = std::max(kChunkBytes, bytes);
            hip_ok(hipHostMalloc((void**)&c.host, c.cap, hipHostMallocDefault), "hipHostMalloc");
            w.chunks.push_back(c);
        }
        Chunk& c = w.chunks[w.cur];
        if (c.used + bytes <= c.cap) {
            const size_t off = c.used;
            c.used += bytes;
            return {w.cur, off};
        }
    }
}

Batch& batch_for(aeon_hip_stager* s, Window& w, void* out)
{
    for (auto& b : w.batches)
        if (b->out == out) return *b;
    auto b  = std::make_unique<Batch>();
    b->out  = out;
    b->descs.resize(s->batch);
    b->params.resize(s->batch);
    b->have.reset(new std::atomic<uint8_t>[s->batch]);
    for (int i = 0; i < s->batch; i++) b->have[i] = 0;
    w.batches.push_back(std::move(b));
    return *w.batches.back();
}

// The window's launch (the first flush / launch): H2D of the pinned chunks, one kernel launch over every
// staged record, then per batch buffer its D2H (or zero-copy stores) and completion event, all on the
// window's stream.  Caller holds s->mu.
void launch_window(aeon_hip_stager* s, Window& w)
{
    size_t total = 0;
    for (Chunk& c : w.chunks) {
        c.base = total;
        total += c.used;
    }
    std::vector<aeon_img_desc>   descs;
    std::vector<aeon_aug_params> params;
    std::vector<void*>           views;
    bool                         all_mapped = true;
    for (auto& bp : w.batches) {
        Batch& b = *bp;
        b.n = 0;
        while (b.n < s->batch && b.have[b.n]) b.n++;
        for (int i = b.n; i < s->batch; i++)
            if (b.have[i]) fail(AEON_HIP_EINVAL, "batch staged with a hole: idx " + std::to_string(b.n) + " missing");
        b.first = (int)descs.size();
        for (int i = 0; i < b.n; i++) {
            aeon_img_desc d = b.descs[i];
            d.offset        = w.chunks[d.offset >> 48].base + (d.offset & ((1ull << 48) - 1));
            descs.push_back(d);
            params.push_back(b.params[i]);
        }
        void* v = (s->kind & AEON_STAGER_DEVICE_OUT) ? nullptr : mapped_view(b.out);
        views.push_back(v);
        all_mapped = all_mapped && v;
    }
    // The window's sources: read by the kernels straight from its pinned chunk over PCIe when the outputs
    // go to pinned host buffers too and the window fits one chunk -- no H2D ahead of the kernels (the
    // runtime may run that copy as a blit kernel, which then cannot overlap the previous window's
    // persistent grid: C2 60 K vs ~80 K records/s, tools/aeon_path_cpp.cpp) -- else one H2D per chunk into
    // the window's device arena.
    const bool on_device = (s->kind & AEON_STAGER_DEVICE_OUT) != 0;
    bool       all_out_mapped = !on_device;
    for (auto& bp : w.batches) all_out_mapped = all_out_mapped && mapped_view(bp->out);
    int         used_chunks = 0;
    const Chunk* used = nullptr; // (its base is 0: the chunks before it hold nothing)
    for (const Chunk& c : w.chunks)
        if (c.used) used_chunks++, used = used ? used : &c;
    static const bool src_copy = [] {
        const char* e = std::getenv("AEON_HIP_STAGER_SRC_COPY");
        return e && std::atoi(e) != 0;
    }();
    const uint8_t* src_base = nullptr;
    if (all_out_mapped && used_chunks == 1 && !src_copy) src_base = (const uint8_t*)mapped_view(used->host);
    if (!src_base) {
        grow(w.dev_src, w.dev_src_cap, std::max<size_t>(total, 16));
        for (const Chunk& c : w.chunks)
            if (c.used)
                hip_ok(hipMemcpyAsync(w.dev_src + c.base, c.host, c.used, hipMemcpyHostToDevice, w.stream),
                       "hipMemcpyAsync");
        src_base = w.dev_src;
    }
    const size_t item = s->out.item_stride;
    auto run = [&](int first, int n, void* dst) {
        if (n == 0) return;
        if ((s->kind & ~AEON_STAGER_DEVICE_OUT) == AEON_STAGER_MASK)
            abi_ok(aeon_hip_mask_batch(s->ctx, n, descs.data() + first, src_base, params.data() + first, &s->out,
                                       dst, w.stream));
        else
            abi_ok(aeon_hip_augment_batch(s->ctx, n, descs.data() + first, src_base, params.data() + first, &s->out,
                                          dst, w.stream));
    };
    if (on_device || all_mapped) {
        // outputs the kernels can store into directly (device batch buffers, or pinned host ones over
        // PCIe): one launch per batch, queued back to back
        for (size_t k = 0; k < w.batches.size(); k++) {
            Batch& b = *w.batches[k];
            run(b.first, b.n, on_device ? b.out : views[k]);
            hip_ok(hipEventRecord(b.done, w.stream), "hipEventRecord");
        }
    } else {
        // pageable host batches: the whole window in ONE launch into device memory; each batch's D2H is
        // made by its wait (the consumer's thread): a copy into pageable memory holds the calling thread
        // until the data is out (the runtime stages it), and on the decode thread that made the
        // launch-only post_process wait for the window's kernels (overlap measured below flush)
        grow(w.dev_out, w.dev_out_cap, std::max<size_t>(descs.size() * item, 16));
        run(0, (int)descs.size(), w.dev_out);
        hip_ok(hipEventRecord(w.batches.front()->done, w.stream), "hipEventRecord");
        for (auto& bp : w.batches) {
            Batch& b = *bp;
            if (&b != w.batches.front().get()) hip_ok(hipEventRecord(b.done, w.stream), "hipEventRecord");
            b.d2h = b.n > 0;
        }
    }
    hip_ok(hipEventRecord(w.done, w.stream), "hipEventRecord");
    w.state    = Window::LAUNCHED;
    w.gen      = ++s->gens;
    w.unwaited = (int)w.batches.size();
    std::lock_guard<std::mutex> r(g_reg_mu);
    for (auto& b : w.batches) g_pending[b->out] = Pending{s, w.gen};
}

// Launch the staging window if batch_out belongs to it (the first post_process of a window); mark
// batch_out launched.  Caller holds s->mu.
void launch_for(aeon_hip_stager* s, void* batch_out)
{
    hip_ok(hipSetDevice(s->device), "hipSetDevice");
    Window& sw = s->win[s->cur];
    if (sw.state == Window::STAGING) {
        bool mine = false;
        for (auto& b : sw.batches) mine = mine || b->out == batch_out;
        if (mine) {
            try {
                launch_window(s, sw);
            } catch (...) { // nothing of this window is delivered: drop it whole
                (void)hipStreamSynchronize(sw.stream);
                sw.state = Window::STAGING; // (never registered)
                reset_window(s, sw);
                throw;
            }
        }
    }
    for (Window& w : s->win) {
        if (w.state != Window::LAUNCHED) continue;
        for (auto& b : w.batches)
            if (b->out == batch_out && !b->waited) {
                if (b->launched) fail(AEON_HIP_EINVAL, "batch buffer flushed twice in one window");
                b->launched = true;
                return;
            }
    }
    fail(AEON_HIP_EINVAL, "no records of this window were staged for this batch buffer");
}

// Wait until batch_out's outputs are complete.  found = false: no launched window holds it (nothing to
// wait for).  The window's last wait checks the device error word and retires the window -- unless it
// was dropped and reused meanwhile (its generation changed).
void wait_batch(aeon_hip_stager* s, void* batch_out, bool& found)
{
    hipEvent_t ev = nullptr, wdone = nullptr;
    hipStream_t wstream = nullptr;
    Window*     wp  = nullptr;
    uint64_t    gen = 0;
    bool        last = false;
    void*       copy_dst = nullptr; // pageable batch: its D2H, made here
    const void* copy_src = nullptr;
    size_t      copy_bytes = 0;
    {
        std::lock_guard<std::mutex> l(s->mu);
        for (Window& w : s->win) {
            if (w.state != Window::LAUNCHED || ev) continue;
            for (auto& b : w.batches)
                if (b->out == batch_out && !b->waited) {
                    b->waited = true;
                    ev        = b->done;
                    wp = &w, gen = w.gen, wdone = w.done, wstream = w.stream;
                    last = --w.unwaited == 0;
                    if (b->d2h) {
                        w.copying.fetch_add(1, std::memory_order_acq_rel);
                        copy_dst   = b->out;
                        copy_src   = w.dev_out + (size_t)b->first * s->out.item_stride;
                        copy_bytes = (size_t)b->n * s->out.item_stride;
                    }
                    break;
                }
        }
    }
    found = ev != nullptr;
    if (!found) return;
    hip_ok(hipSetDevice(s->device), "hipSetDevice");
    hip_ok(hipEventSynchronize(ev), "hipEventSynchronize");
    // (the window's device outputs stay until its last wait has returned: reset_window runs after it)
    if (copy_bytes) {
        const hipError_t e = hipMemcpy(copy_dst, copy_src, copy_bytes, hipMemcpyDeviceToHost);
        wp->copying.fetch_sub(1, std::memory_order_acq_rel);
        hip_ok(e, "hipMemcpy");
    }
    if (!last) return;
    while (wp->copying.load(std::memory_order_acquire) != 0) std::this_thread::yield(); // (other batches' copies)
    // the window is complete: surface a device error word, then free it for the window after next
    hip_ok(hipEventSynchronize(wdone), "hipEventSynchronize");
    const int rc = aeon_hip_synchronize(s->ctx, wstream);
    {
        std::lock_guard<std::mutex> l(s->mu);
        if (wp->state == Window::LAUNCHED && wp->gen == gen) reset_window(s, *wp);
    }
    abi_ok(rc);
}

} // namespace

extern "C" {

int aeon_hip_stager_create(aeon_hip_ctx* ctx, int kind, const aeon_out_desc* out, int batch_size,
                           aeon_hip_stager** result)
{
    return stager_guarded([&] {
        if (!ctx || !out || !result) fail(AEON_HIP_EINVAL, "null argument");
        if (batch_size <= 0) fail(AEON_HIP_EINVAL, "batch_size must be > 0");
        const int base = kind & ~AEON_STAGER_DEVICE_OUT;
        if (base != AEON_STAGER_IMAGE && base != AEON_STAGER_MASK) fail(AEON_HIP_EINVAL, "unknown stager kind");
        if (out->item_stride == 0) fail(AEON_HIP_EINVAL, "out->item_stride is 0");
        auto s   = std::make_unique<aeon_hip_stager>();
        s->ctx   = ctx;
        s->kind  = kind;
        s->out   = *out;
        s->batch = batch_size;
        hip_ok(hipGetDevice(&s->device), "hipGetDevice");
        for (Window& w : s->win) {
            hip_ok(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking), "hipStreamCreate");
            hip_ok(hipEventCreateWithFlags(&w.done, hipEventDisableTiming), "hipEventCreate");
        }
        *result = s.release();
    });
}

int aeon_hip_stager_destroy(aeon_hip_stager* s)
{
    if (!s) return 0;
    {
        // no new consumer wait can find this stager once its buffers are unregistered; the ones already
        // inside it finish first
        std::lock_guard<std::mutex> r(g_reg_mu);
        for (auto it = g_pending.begin(); it != g_pending.end();)
            it = it->second.s == s ? g_pending.erase(it) : std::next(it);
    }
    while (s->waiters.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    (void)hipSetDevice(s->device);
    {
        std::lock_guard<std::mutex> l(s->mu);
        for (Window& w : s->win) {
            if (w.state == Window::LAUNCHED) (void)hipEventSynchronize(w.done);
            if (w.stream) (void)aeon_hip_release_stream(s->ctx, w.stream); // (before the stream goes)
            reset_window(s, w);
            for (Chunk& c : w.chunks) (void)hipHostFree(c.host);
            if (w.dev_src) (void)hipFree(w.dev_src);
            if (w.dev_out) (void)hipFree(w.dev_out);
            if (w.done) (void)hipEventDestroy(w.done);
            if (w.stream) (void)hipStreamDestroy(w.stream);
        }
        for (hipEvent_t e : s->spare_events) (void)hipEventDestroy(e);
        s->spare_events.clear();
    }
    delete s;
    return 0;
}

int aeon_hip_stager_stage(aeon_hip_stager* s, void* batch_out, int idx, const void* pixels, int width, int height,
                          int stride, int channels, int elem_bytes, const aeon_aug_params* params)
{
    return stager_guarded([&] {
        if (!s || !batch_out || !pixels || !params) fail(AEON_HIP_EINVAL, "null argument");
        if (idx < 0 || idx >= s->batch) fail(AEON_HIP_EINVAL, "idx out of range of the batch");
        if (width <= 0 || height <= 0) fail(AEON_HIP_EINVAL, "received an image with size 0, at idx " + std::to_string(idx));
        if (channels != 1 && channels != 3) fail(AEON_HIP_EINVAL, "channels must be 1 or 3");
        if (elem_bytes == 0) elem_bytes = 1;
        if (elem_bytes != 1 && elem_bytes != 2) fail(AEON_HIP_EINVAL, "elem_bytes must be 1 or 2");
        const size_t row = (size_t)width * channels * elem_bytes;
        if (stride == 0) stride = (int)row;
        if ((size_t)stride < row) fail(AEON_HIP_EINVAL, "stride < width * channels * elem_bytes");
        Batch*   b;
        uint8_t* dst;
        size_t   tag;
        {
            std::lock_guard<std::mutex> l(s->mu);
            Window& w = staging_window(s);
            w.state   = Window::STAGING;
            b         = &batch_for(s, w, batch_out);
            if (!b->done) {
                if (!s->spare_events.empty()) {
                    b->done = s->spare_events.back();
                    s->spare_events.pop_back();
                } else {
                    hip_ok(hipSetDevice(s->device), "hipSetDevice");
                    hip_ok(hipEventCreateWithFlags(&b->done, hipEventDisableTiming), "hipEventCreate");
                }
            }
            if (b->have[idx]) fail(AEON_HIP_EINVAL, "idx " + std::to_string(idx) + " staged twice for one batch");
            const auto r = reserve(w, row * height);
            dst          = w.chunks[r.first].host + r.second;
            tag          = ((size_t)r.first << 48) | r.second;
        }
        // the copy itself runs unlocked, on the calling pool thread (the window cannot launch before
        // this provide() returns: aeon flushes after its pool run)
        if ((size_t)stride == row) std::memcpy(dst, pixels, row * height);
        else
            for (int y = 0; y < height; y++) std::memcpy(dst + y * row, (const uint8_t*)pixels + (size_t)y * stride, row);
        b->descs[idx]  = aeon_img_desc{tag, width, height, (int32_t)row, channels, elem_bytes, 0};
        b->params[idx] = *params;
        b->have[idx].store(1, std::memory_order_release);
    });
}

int aeon_hip_stager_launch(aeon_hip_stager* s, void* batch_out)
{
    return stager_guarded([&] {
        if (!s || !batch_out) fail(AEON_HIP_EINVAL, "null argument");
        std::lock_guard<std::mutex> l(s->mu);
        launch_for(s, batch_out);
    });
}

int aeon_hip_stager_wait(aeon_hip_stager* s, void* batch_out)
{
    return stager_guarded([&] {
        if (!batch_out) fail(AEON_HIP_EINVAL, "null argument");
        if (!s) { // the consumer's form: whichever stager launched this buffer, if any
            {
                // the stager is pinned (waiters) under the registry lock, which its destroy takes to
                // unregister: it cannot go away between the lookup and the wait
                std::lock_guard<std::mutex> r(g_reg_mu);
                auto it = g_pending.find(batch_out);
                if (it == g_pending.end()) return;
                s = it->second.s;
                s->waiters.fetch_add(1, std::memory_order_acq_rel);
            }
            struct Unpin {
                aeon_hip_stager* s;
                ~Unpin() { s->waiters.fetch_sub(1, std::memory_order_acq_rel); }
            } unpin{s};
            bool found = false;
            wait_batch(s, batch_out, found);
            return;
        }
        bool found = false;
        wait_batch(s, batch_out, found);
    });
}

int aeon_hip_stager_flush(aeon_hip_stager* s, void* batch_out)
{
    return stager_guarded([&] {
        if (!s || !batch_out) fail(AEON_HIP_EINVAL, "null argument");
        {
            std::lock_guard<std::mutex> l(s->mu);
            launch_for(s, batch_out);
        }
        bool found = false;
        wait_batch(s, batch_out, found);
        if (!found) fail(AEON_HIP_EINVAL, "batch buffer completed by another thread's wait");
    });
}

const char* aeon_hip_stager_last_error(void) { return g_stager_err.c_str(); }

} // extern "C"
