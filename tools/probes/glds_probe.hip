// LDS-DMA probe: buffer_load_dword{,x3,x4} ... lds -- exact bytes at byte-unaligned offsets, 0 for an
// access crossing num_records or far out of range, and the LDS placement of wide loads (lane*size?).
// (development only)
#include <hip/hip_runtime.h>
#include <stdint.h>
extern "C" __global__ __launch_bounds__(64) void probe_glds(const uint8_t* src, uint32_t* out, int nbytes, int base,
                                                            int far, int size)
{
    __shared__ uint32_t lds[64 * 4];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = 0xdeadbeef;
    __syncthreads();
    auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nbytes, 0x00020000);
    int off = base + (size == 4 ? 3 : size) * threadIdx.x;
    if (far && threadIdx.x == 5) off = 0x7ffffff0;
    uint32_t m0 = (uint32_t)(size_t)(__attribute__((address_space(3))) uint32_t*)lds;
    if (size == 4)
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(rs) : "memory");
    else if (size == 12)
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx3 %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(rs) : "memory");
    else
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(rs) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) out[i] = lds[i];
}
extern "C" void launch(const uint8_t* src, uint32_t* out, int nbytes, int base, int far, int size)
{
    hipLaunchKernelGGL(probe_glds, dim3(1), dim3(64), 0, 0, src, out, nbytes, base, far, size);
}
