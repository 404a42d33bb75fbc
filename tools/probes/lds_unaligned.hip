// Probe: ds_read_b32 / ds_read_b64 at byte-unaligned LDS addresses (development only).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
extern "C" __global__ __launch_bounds__(64) void probe_lds(uint32_t* out, int stride)
{
    __shared__ uint32_t lds[512];
    for (int i = threadIdx.x; i < 512; i += 64) lds[i] = (4 * i) | ((4 * i + 1) << 8) | ((4 * i + 2) << 16) | ((4 * i + 3) << 24);
    __syncthreads();
    const uint32_t base = (uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t*)lds;
    const uint32_t a    = base + stride * threadIdx.x + 1;
    uint32_t v32 = *(__attribute__((address_space(3))) uint32_t*)(size_t)a;
    u32x2 v64    = *(__attribute__((address_space(3))) u32x2*)(size_t)a;
    out[threadIdx.x * 3 + 0] = v32;
    out[threadIdx.x * 3 + 1] = v64.x;
    out[threadIdx.x * 3 + 2] = v64.y;
}
extern "C" void launch(uint32_t* out, int stride)
{
    hipLaunchKernelGGL(probe_lds, dim3(1), dim3(64), 0, 0, out, stride);
}
