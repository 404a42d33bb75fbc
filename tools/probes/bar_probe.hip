// Can the host write job tables straight into device-local (VRAM) memory?  Allocates fine-grained /
// uncached device memory, writes it from the CPU (through the PCIe BAR), times that, and has a
// kernel read it back.  Development probe (tools/probes), not part of the library.
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void sum_words(const uint32_t* p, int n, uint32_t* out)
{
    uint32_t s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    atomicAdd(out, s);
}

int main()
{
    const int      n = 16384; // 64 KB
    const unsigned flags[2] = {hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    const char*    names[2] = {"finegrained", "uncached"};
    uint32_t*      out;
    hipMalloc(&out, 4);
    std::vector<uint32_t> src(n);
    for (int i = 0; i < n; i++) src[i] = i * 2654435761u;
    uint32_t want = 0;
    for (int i = 0; i < n; i++) want += src[i];
    for (int f = 0; f < 2; f++) {
        uint32_t* d = nullptr;
        hipError_t e = hipExtMallocWithFlags((void**)&d, n * 4, flags[f]);
        printf("%s: alloc %s\n", names[f], hipGetErrorString(e));
        if (e != hipSuccess) continue;
        hipPointerAttribute_t attr;
        e = hipPointerGetAttributes(&attr, d);
        printf("  attr %s type %d hostPointer %p devicePointer %p\n", hipGetErrorString(e), (int)attr.type, attr.hostPointer,
               attr.devicePointer);
        fflush(stdout);
        double best = 1e9;
        for (int r = 0; r < 5; r++) {
            auto t0 = std::chrono::steady_clock::now();
            std::memcpy(d, src.data(), n * 4); // CPU writes to the device pointer
            std::atomic_thread_fence(std::memory_order_seq_cst);
            auto t1 = std::chrono::steady_clock::now();
            best = std::min(best, std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        printf("  CPU memcpy 64 KB into it: %.2f us\n", best);
        hipMemset(out, 0, 4);
        sum_words<<<1, 256>>>(d, n, out);
        uint32_t got = 0;
        hipMemcpy(&got, out, 4, hipMemcpyDeviceToHost);
        printf("  kernel read back: %s\n", got == want ? "ok" : "MISMATCH");
        hipFree(d);
    }
    return 0;
}
