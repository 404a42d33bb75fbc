// CU-partition probe: how much HBM bandwidth a pass-2-like stream (read u8, write 4x f32) gets
// from n CUs of a CU-masked stream, and whether a VALU-bound kernel on the complementary CUs runs
// beside it undisturbed.  Development only:  hipcc --offload-arch=gfx950 -O3 cumask_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include <unistd.h>

#define CK(x)                                                                                       \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 1 B read : 4 B written per element, like contrast pass 2 (u8 intermediate -> f32 CHW)
__global__ __launch_bounds__(256) void expand_u8(const uint32_t* __restrict__ src, f32x4* __restrict__ dst, size_t n4)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t w = __builtin_nontemporal_load(src + i);
        f32x4 v = {(float)(w & 255) * 0.5f, (float)((w >> 8) & 255) * 0.5f, (float)((w >> 16) & 255) * 0.5f,
                   (float)(w >> 24) * 0.5f};
        __builtin_nontemporal_store(v, dst + i);
    }
}

// VALU-bound stand-in for contrast pass 1: a fixed integer chain per lane
__global__ __launch_bounds__(256) void valu_spin(uint32_t* out, int iters)
{
    uint32_t a = threadIdx.x, b = blockIdx.x | 1;
    for (int k = 0; k < iters; k++) {
        a = a * 1664525u + b;
        b = (b ^ (a >> 7)) + 0x9e3779b9u;
    }
    if (a == 0x12345678u && b == 0) out[0] = a; // keep the chain live
}

static std::vector<uint32_t> mask_of(int n_cu, int n, int stride_mode, bool complement)
{
    std::vector<uint32_t> m((n_cu + 31) / 32, 0);
    for (int c = 0; c < n_cu; c++) {
        // n/8 CUs of every 32: balanced over the 8 XCDs whether the mask's bit c maps to XCD c/32 or
        // c%8 (a mask that leaves an XCD without CUs never finishes a dispatch)
        bool on = (c % 32) < n / 8;
        (void)stride_mode;
        if (complement) on = !on;
        if (on) m[c / 32] |= 1u << (c % 32);
    }
    return m;
}

// hipEventSynchronize with a deadline: a dispatch that cannot run ends the probe
static void wait_or_die(hipEvent_t e)
{
    for (int i = 0; i < 3000; i++) {
        hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) CK(q);
        usleep(1000);
    }
    std::printf("HUNG: event not reached in 3 s\n");
    std::exit(3);
}

int main()
{
    setvbuf(stdout, nullptr, _IONBF, 0);
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int n_cu = p.multiProcessorCount;
    std::printf("CUs %d  %s\n", n_cu, p.gcnArchName);
    const size_t bytes_in = 154ull << 20, n4 = bytes_in / 4;
    uint32_t* src;
    f32x4*    dst;
    uint32_t* junk;
    CK(hipMalloc(&src, bytes_in));
    CK(hipMalloc(&dst, n4 * sizeof(f32x4)));
    CK(hipMalloc(&junk, 64));
    CK(hipMemset(src, 1, bytes_in));
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    CK(hipEventCreate(&e3));
    const double moved = bytes_in * 5.0;
    const int    spin  = 5000;
    for (int stride_mode = 0; stride_mode < 1; stride_mode++) {
        for (int n : {16, 32, 48, 64, 96, 128, 256}) {
            if (n > n_cu) continue;
            auto        mB = mask_of(n_cu, n, stride_mode, false);
            auto        mA = mask_of(n_cu, n, stride_mode, true);
            hipStream_t sB, sA;
            CK(hipExtStreamCreateWithCUMask(&sB, (uint32_t)mB.size(), mB.data()));
            const bool have_a = n < n_cu;
            if (have_a) CK(hipExtStreamCreateWithCUMask(&sA, (uint32_t)mA.size(), mA.data()));
            // bandwidth alone on n CUs
            hipLaunchKernelGGL(expand_u8, dim3(n * 8), dim3(256), 0, sB, src, dst, n4);
            CK(hipEventRecord(e0, sB));
            for (int r = 0; r < 5; r++) hipLaunchKernelGGL(expand_u8, dim3(n * 8), dim3(256), 0, sB, src, dst, n4);
            CK(hipEventRecord(e1, sB));
            wait_or_die(e1);
            float ms_b = 0;
            CK(hipEventElapsedTime(&ms_b, e0, e1));
            ms_b /= 5;
            float ms_a = 0, ms_ab = 0, ms_ba = 0;
            if (have_a) {
                // VALU kernel alone on the other CUs, then both together
                CK(hipEventRecord(e2, sA));
                hipLaunchKernelGGL(valu_spin, dim3((n_cu - n) * 8), dim3(256), 0, sA, junk, spin);
                CK(hipEventRecord(e3, sA));
                wait_or_die(e3);
                CK(hipEventElapsedTime(&ms_a, e2, e3));
                CK(hipEventRecord(e2, sA));
                CK(hipEventRecord(e0, sB));
                hipLaunchKernelGGL(valu_spin, dim3((n_cu - n) * 8), dim3(256), 0, sA, junk, spin);
                for (int r = 0; r < 5; r++) hipLaunchKernelGGL(expand_u8, dim3(n * 8), dim3(256), 0, sB, src, dst, n4);
                CK(hipEventRecord(e3, sA));
                CK(hipEventRecord(e1, sB));
                wait_or_die(e3);
                wait_or_die(e1);
                CK(hipEventElapsedTime(&ms_ab, e2, e3));
                CK(hipEventElapsedTime(&ms_ba, e0, e1));
            }
            std::printf("%s n=%3d  expand alone %7.1f us (%5.2f TB/s)  | valu alone on %3d CUs %8.1f us, together: valu %8.1f us, "
                        "expand x5 %8.1f us\n",
                        "balanced", n, ms_b * 1e3, moved / (ms_b * 1e-3) / 1e12, n_cu - n,
                        ms_a * 1e3, ms_ab * 1e3, ms_ba * 1e3);
            CK(hipStreamDestroy(sB));
            if (have_a) CK(hipStreamDestroy(sA));
        }
    }
    return 0;
}
