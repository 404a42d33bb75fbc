// stager.cpp -- the aeon-side drop-in's staging + window flush (aeon_hip_stager_*, include/aeon_hip.h).
//
// aeon runs provide(idx, record, out_buf) for every record of a decode window on its pool and then
// (the one-line change) post_process(out_buf) once per batch of the window
// (src/batch_decoder.cpp:62-99).  A stager is what provider::image / provider::pixelmask hold to make
// those two calls the GPU path:
//   stage(batch_out, idx, pixels, params)  -- provide(): the decoded record's bytes into pinned memory
//                                            (lock-free bump allocation in pinned chunks; concurrent)
//   flush(batch_out)                       -- post_process(): the FIRST flush after a window's stages
//                                            launches the whole window -- one H2D per pinned chunk, ONE
//                                            augment (or mask) launch over every staged record of every
//                                            batch, one D2H per batch buffer (or, for pinned batch
//                                            buffers, the kernels store into them directly) -- and
//                                            every flush waits only for its own batch's output.
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
    bool       flushed = false;
};

} // namespace

struct aeon_hip_stager {
    aeon_hip_ctx* ctx   = nullptr;
    int           kind  = AEON_STAGER_IMAGE;
    aeon_out_desc out{};
    int           batch = 0;
    int           device = 0;
    hipStream_t   stream = nullptr;
    std::mutex    mu;
    std::vector<Chunk>                  chunks;
    int                                 cur = 0; // chunk being filled
    std::vector<std::unique_ptr<Batch>> batches; // this window's, in first-stage order
    std::vector<hipEvent_t>             spare_events;
    bool          launched = false;
    int           unflushed = 0;
    hipEvent_t    window_done = nullptr;
    uint8_t*      dev_src = nullptr;
    size_t        dev_src_cap = 0;
    uint8_t*      dev_out = nullptr;
    size_t        dev_out_cap = 0;
};

namespace {

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
    if (p) hip_ok(hipFree(p), "hipFree");
    p = nullptr, cap = 0;
    const size_t n = std::max(need, cap + cap / 2);
    hip_ok(hipMalloc((void**)&p, n), "hipMalloc");
    cap = n;
}

// Forget the completed window: batches gone, chunks empty (their memory is kept).
void reset_window(aeon_hip_stager* s)
{
    for (auto& b : s->batches)
        if (b->done) s->spare_events.push_back(b->done);
    s->batches.clear();
    for (Chunk& c : s->chunks) c.used = 0;
    s->cur       = 0;
    s->launched  = false;
    s->unflushed = 0;
}

// Reserve `bytes` (16-aligned) of pinned staging: returns (chunk, offset).  Caller holds s->mu.
std::pair<int, size_t> reserve(aeon_hip_stager* s, size_t bytes)
{
    bytes = (bytes + 15) & ~(size_t)15;
    for (;; s->cur++) {
        if (s->cur == (int)s->chunks.size()) {
            Chunk c;
            c.cap = std::max(kChunkBytes, bytes);
            hip_ok(hipHostMalloc((void**)&c.host, c.cap, hipHostMallocDefault), "hipHostMalloc");
            s->chunks.push_back(c);
        }
        Chunk& c = s->chunks[s->cur];
        if (c.used + bytes <= c.cap) {
            const size_t off = c.used;
            c.used += bytes;
            return {s->cur, off};
        }
    }
}

Batch& batch_for(aeon_hip_stager* s, void* out)
{
    for (auto& b : s->batches)
        if (b->out == out) return *b;
    auto b  = std::make_unique<Batch>();
    b->out  = out;
    b->descs.resize(s->batch);
    b->params.resize(s->batch);
    b->have.reset(new std::atomic<uint8_t>[s->batch]);
    for (int i = 0; i < s->batch; i++) b->have[i] = 0;
    s->batches.push_back(std::move(b));
    return *s->batches.back();
}

// The window's launch (the first flush): H2D of the pinned chunks, one kernel launch over every
// staged record, then per batch buffer its D2H (or zero-copy stores) and completion event.
void launch_window(aeon_hip_stager* s)
{
    size_t total = 0;
    for (Chunk& c : s->chunks) {
        c.base = total;
        total += c.used;
    }
    grow(s->dev_src, s->dev_src_cap, std::max<size_t>(total, 16));
    for (const Chunk& c : s->chunks)
        if (c.used)
            hip_ok(hipMemcpyAsync(s->dev_src + c.base, c.host, c.used, hipMemcpyHostToDevice, s->stream),
                   "hipMemcpyAsync");
    std::vector<aeon_img_desc>   descs;
    std::vector<aeon_aug_params> params;
    std::vector<void*>           views;
    bool                         all_mapped = true;
    for (auto& bp : s->batches) {
        Batch& b = *bp;
        b.n = 0;
        while (b.n < s->batch && b.have[b.n]) b.n++;
        for (int i = b.n; i < s->batch; i++)
            if (b.have[i]) fail(AEON_HIP_EINVAL, "batch staged with a hole: idx " + std::to_string(b.n) + " missing");
        b.first = (int)descs.size();
        for (int i = 0; i < b.n; i++) {
            aeon_img_desc d = b.descs[i];
            d.offset        = s->chunks[d.offset >> 48].base + (d.offset & ((1ull << 48) - 1));
            descs.push_back(d);
            params.push_back(b.params[i]);
        }
        void* v = (s->kind & AEON_STAGER_DEVICE_OUT) ? nullptr : mapped_view(b.out);
        views.push_back(v);
        all_mapped = all_mapped && v;
    }
    const size_t item = s->out.item_stride;
    auto run = [&](int first, int n, void* dst) {
        if (n == 0) return;
        if ((s->kind & ~AEON_STAGER_DEVICE_OUT) == AEON_STAGER_MASK)
            abi_ok(aeon_hip_mask_batch(s->ctx, n, descs.data() + first, s->dev_src, params.data() + first, &s->out,
                                       dst, s->stream));
        else
            abi_ok(aeon_hip_augment_batch(s->ctx, n, descs.data() + first, s->dev_src, params.data() + first, &s->out,
                                          dst, s->stream));
    };
    const bool on_device = (s->kind & AEON_STAGER_DEVICE_OUT) != 0;
    if (on_device || all_mapped) {
        // outputs the kernels can store into directly (device batch buffers, or pinned host ones over
        // PCIe): one launch per batch, queued back to back
        for (size_t k = 0; k < s->batches.size(); k++) {
            Batch& b = *s->batches[k];
            run(b.first, b.n, on_device ? b.out : views[k]);
            hip_ok(hipEventRecord(b.done, s->stream), "hipEventRecord");
        }
    } else {
        // pageable host batches: the whole window in ONE launch into device memory, then a D2H into
        // each batch buffer
        grow(s->dev_out, s->dev_out_cap, std::max<size_t>(descs.size() * item, 16));
        run(0, (int)descs.size(), s->dev_out);
        for (auto& bp : s->batches) {
            Batch& b = *bp;
            if (b.n)
                hip_ok(hipMemcpyAsync(b.out, s->dev_out + (size_t)b.first * item, (size_t)b.n * item,
                                      hipMemcpyDeviceToHost, s->stream),
                       "hipMemcpyAsync");
            hip_ok(hipEventRecord(b.done, s->stream), "hipEventRecord");
        }
    }
    hip_ok(hipEventRecord(s->window_done, s->stream), "hipEventRecord");
    s->launched  = true;
    s->unflushed = (int)s->batches.size();
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
        hip_ok(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking), "hipStreamCreate");
        hip_ok(hipEventCreateWithFlags(&s->window_done, hipEventDisableTiming), "hipEventCreate");
        *result = s.release();
    });
}

int aeon_hip_stager_destroy(aeon_hip_stager* s)
{
    if (!s) return 0;
    (void)hipSetDevice(s->device);
    if (s->launched) (void)hipEventSynchronize(s->window_done);
    reset_window(s);
    for (hipEvent_t e : s->spare_events) (void)hipEventDestroy(e);
    for (Chunk& c : s->chunks) (void)hipHostFree(c.host);
    if (s->dev_src) (void)hipFree(s->dev_src);
    if (s->dev_out) (void)hipFree(s->dev_out);
    if (s->window_done) (void)hipEventDestroy(s->window_done);
    if (s->stream) (void)hipStreamDestroy(s->stream);
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
            if (s->launched) { // the previous window (some batch never flushed): let it finish, start anew
                hip_ok(hipSetDevice(s->device), "hipSetDevice");
                hip_ok(hipEventSynchronize(s->window_done), "hipEventSynchronize");
                reset_window(s);
            }
            b = &batch_for(s, batch_out);
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
            const auto r = reserve(s, row * height);
            dst          = s->chunks[r.first].host + r.second;
            tag          = ((size_t)r.first << 48) | r.second;
        }
        // the copy itself runs unlocked, on the calling pool thread
        if ((size_t)stride == row) std::memcpy(dst, pixels, row * height);
        else
            for (int y = 0; y < height; y++) std::memcpy(dst + y * row, (const uint8_t*)pixels + (size_t)y * stride, row);
        b->descs[idx]  = aeon_img_desc{tag, width, height, (int32_t)row, channels, elem_bytes, 0};
        b->params[idx] = *params;
        b->have[idx].store(1, std::memory_order_release);
    });
}

int aeon_hip_stager_flush(aeon_hip_stager* s, void* batch_out)
{
    return stager_guarded([&] {
        if (!s || !batch_out) fail(AEON_HIP_EINVAL, "null argument");
        hipEvent_t ev   = nullptr;
        bool       last = false;
        {
            std::lock_guard<std::mutex> l(s->mu);
            hip_ok(hipSetDevice(s->device), "hipSetDevice");
            if (!s->launched) {
                if (s->batches.empty()) fail(AEON_HIP_EINVAL, "flush without staged records");
                try {
                    launch_window(s);
                } catch (...) { // nothing of this window is delivered: drop it whole
                    (void)hipStreamSynchronize(s->stream);
                    reset_window(s);
                    throw;
                }
            }
            Batch* b = nullptr;
            for (auto& bp : s->batches)
                if (bp->out == batch_out) b = bp.get();
            if (!b) fail(AEON_HIP_EINVAL, "no records of this window were staged for this batch buffer");
            if (b->flushed) fail(AEON_HIP_EINVAL, "batch buffer flushed twice in one window");
            b->flushed = true;
            ev         = b->done;
            last       = --s->unflushed == 0;
        }
        hip_ok(hipEventSynchronize(ev), "hipEventSynchronize");
        if (last) {
            // the window is complete: surface a device error word, then take the next window's stages
            const int rc = aeon_hip_synchronize(s->ctx, s->stream);
            {
                std::lock_guard<std::mutex> l(s->mu);
                reset_window(s);
            }
            abi_ok(rc);
        }
    });
}

const char* aeon_hip_stager_last_error(void) { return g_stager_err.c_str(); }

} // extern "C"
