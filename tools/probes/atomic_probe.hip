// Development probe: latency/throughput of device-scope atomics used as a work counter.
// Each workgroup's lane 0 takes `k` tickets from counter (blockIdx % spread) * 64 words apart,
// each dependent on the previous one; out[w] = sum of tickets (keeps the atomics live).
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void ticket_k(uint32_t* ctr, uint32_t* out, int k, int spread, int spin)
{
    if (threadIdx.x != 0) return;
    uint32_t acc = 0;
    uint32_t* c = ctr + (blockIdx.x % spread) * 64;
    for (int i = 0; i < k; i++) {
        const uint32_t v = atomicAdd(c + (acc & 0), 1u);
        acc += v;
        if (out) out[8192 + blockIdx.x * k + i] = v;
        for (int s = 0; s < spin; s++) __builtin_amdgcn_s_sleep(127);
    }
    out[blockIdx.x] = acc;
}

extern "C" int ticket_launch(uint32_t* ctr, uint32_t* out, int grid, int threads, int k, int spread, int spin,
                             hipStream_t s)
{
    hipLaunchKernelGGL(ticket_k, dim3(grid), dim3(threads), 0, s, ctr, out, k, spread, spin);
    return (int)hipGetLastError();
}
