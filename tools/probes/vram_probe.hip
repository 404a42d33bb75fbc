// Probe: can the host write a small per-call table straight into device memory (fine-grained VRAM
// over the PCIe BAR), and how long does a 16-workgroup kernel take to read 37 KB of it, compared
// with reading the same bytes from pinned host memory (system-coherent loads, as plan_records does)?
// Build: hipcc --offload-arch=gfx950 -O2 vram_probe.hip -o vram_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int AUX>
__global__ __launch_bounds__(128) void read_table(const u32x4* src, int n16, uint32_t* out)
{
    __shared__ uint32_t acc[128];
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, n16 * 16, 0x00020000);
    uint32_t   s  = 0;
    for (int i = blockIdx.x * 128 + threadIdx.x; i < n16; i += gridDim.x * 128) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, i * 16, 0, AUX);
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    acc[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int k = 0; k < 128; k++) t ^= acc[k];
        out[blockIdx.x] = t;
    }
}

int main()
{
    const size_t bytes = 256 * 144; // 256 PlanRecords
    const int    n16   = (int)(bytes / 16);
    void*        fg    = nullptr;
    CHECK(hipExtMallocWithFlags(&fg, bytes, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at{};
    CHECK(hipPointerGetAttributes(&at, fg));
    std::printf("fine-grained VRAM: device %p host view %p type %d\n", at.devicePointer, at.hostPointer, (int)at.type);
    void* pinned = nullptr;
    CHECK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    void* pinned_dev = nullptr;
    CHECK(hipHostGetDevicePointer(&pinned_dev, pinned, 0));
    uint32_t* out = nullptr;
    CHECK(hipMalloc((void**)&out, 64 * 4));
    std::vector<uint8_t> h(bytes);
    for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)(i * 131 + 7);
    std::memcpy(pinned, h.data(), bytes);
    const bool host_view = at.hostPointer != nullptr;
    if (host_view) std::memcpy(at.hostPointer, h.data(), bytes);
    else CHECK(hipMemcpy(fg, h.data(), bytes, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto time = [&](const char* what, auto launch) -> int {
        for (int w = 0; w < 20; w++) launch(nullptr, nullptr);
        CHECK(hipDeviceSynchronize());
        float tot = 0;
        for (int r = 0; r < 100; r++) {
            launch(e0, e1);
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            tot += ms;
        }
        uint32_t o[16];
        CHECK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
        uint32_t x = 0;
        for (int k = 0; k < 16; k++) x ^= o[k];
        std::printf("%-34s %.2f us per launch (checksum %08x)\n", what, tot * 1000 / 100, x);
        return 0;
    };
    auto L = [&](auto kern, const void* src) {
        return [=](hipEvent_t a, hipEvent_t b) {
            hipExtLaunchKernel((const void*)kern, dim3(16), dim3(128), nullptr, 0, 0, a, b, 0);
            (void)src;
        };
    };
    (void)L;
    auto run = [&](const char* what, auto kern, const void* src) {
        return time(what, [&](hipEvent_t a, hipEvent_t b) {
            void* args[] = {(void*)&src, (void*)&n16, (void*)&out};
            hipExtLaunchKernel((const void*)kern, dim3(16), dim3(128), args, 0, 0, a, b, 0);
        });
    };
    if (run("pinned host, sc0 sc1 loads", read_table<1 | 16>, pinned_dev)) return 1;
    if (run("fine-grained VRAM, sc0 sc1 loads", read_table<1 | 16>, fg)) return 1;
    if (run("fine-grained VRAM, default loads", read_table<0>, fg)) return 1;
    // host rewrites between launches: visibility of host writes through the BAR view
    if (host_view) {
        for (int r = 0; r < 3; r++) {
            for (size_t i = 0; i < bytes; i++) h[i] = (uint8_t)(i * 7 + r);
            std::memcpy(at.hostPointer, h.data(), bytes);
            std::memcpy(pinned, h.data(), bytes);
            __builtin_ia32_sfence();
            uint32_t a[16], b[16];
            const void* s1 = fg;
            const void* s2 = pinned_dev;
            void* args1[] = {(void*)&s1, (void*)&n16, (void*)&out};
            CHECK(hipLaunchKernel((const void*)read_table<1 | 16>, dim3(16), dim3(128), args1, 0, 0));
            CHECK(hipMemcpy(a, out, sizeof(a), hipMemcpyDeviceToHost));
            void* args2[] = {(void*)&s2, (void*)&n16, (void*)&out};
            CHECK(hipLaunchKernel((const void*)read_table<1 | 16>, dim3(16), dim3(128), args2, 0, 0));
            CHECK(hipMemcpy(b, out, sizeof(b), hipMemcpyDeviceToHost));
            std::printf("rewrite %d: VRAM view %s pinned\n", r, std::memcmp(a, b, sizeof(a)) == 0 ? "==" : "!=");
        }
    }
    return 0;
}
