// probe_kernels.hip -- bandwidth probes shaped like augment_tiles' C2 launch (development only).
// Each "tile" = ROWS output rows of a 224-wide, 3-plane f32 CHW item (one float4 per lane and
// plane per 4-pixel group), like the kernel's OF_F32_CHW_VEC store path.  Variants:
//   0: write-only, one tile per workgroup (grid = tiles)
//   1: write-only, persistent grid-stride over tiles
//   2: load the tile's u8 source footprint (stage-like, 16 B per lane) then write
//   3: like 2, persistent
//   4: like 2, but the tile's source address comes from a 256-byte per-item descriptor loaded
//      first (a dependent round trip, as augment_tiles' job load)
//   5: like 2, plus `work` dependent VALU iterations per lane between the loads and the stores
//   6: 4 + 5
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/probe_kernels.hip -o tools/libprobe.so
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int W = 224, H = 224;

template <int MODE>
__global__ __launch_bounds__(256) void probe(const uint8_t* src, float* out, int n_items, int rows,
                                               int src_item_bytes, int src_tile_bytes, int grid_tiles, int work,
                                               const uint64_t* desc)
{
    const int tiles_per_item = (H + rows - 1) / rows;
    const int total          = n_items * tiles_per_item;
    const bool persistent    = MODE == 1 || MODE == 3;
    const bool load          = MODE >= 2;
    const bool dep           = MODE == 4 || MODE == 6;
    const bool valu          = MODE == 5 || MODE == 6;
    __shared__ u32x4 lds[1024];
    for (int t = blockIdx.x; t < total; t += persistent ? gridDim.x : total) {
        const int item = t / tiles_per_item, tile = t - item * tiles_per_item;
        uint32_t  acc  = 0;
        if (load) {
            const uint8_t* base = dep ? (const uint8_t*)desc[item * 32] : src + (size_t)item * src_item_bytes;
            const auto     rs   = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, src_item_bytes, 0x00020000);
            for (int i = threadIdx.x; i * 16 < src_tile_bytes; i += 256) {
                u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, tile * src_tile_bytes / 2 + i * 16, 0, 0);
                lds[i & 1023] = v;
            }
            __syncthreads();
            acc = lds[threadIdx.x].x & 1;
        }
        if (valu) {
            uint32_t x = acc + threadIdx.x;
            for (int i = 0; i < work; i++) x = (x ^ (x >> 3)) + 0x9e3779b9u; // 3 full-rate VALU ops
            acc = x & 1;
        }
        const int  plane = W * H;
        const auto orsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(out + (size_t)item * 3 * plane), 0,
                                                             3 * plane * 4, 0x00020000);
        const int  y0 = tile * rows, y1 = min(H, y0 + rows);
        const int  gpr = W / 4;
        for (int g = threadIdx.x; g < (y1 - y0) * gpr; g += 256) {
            const int ry = g / gpr, cg = g - ry * gpr;
            const int idx = (y0 + ry) * W + cg * 4;
            u32x4     v   = {(uint32_t)idx + acc, 1u, 2u, 3u};
#pragma unroll
            for (int c = 0; c < 3; c++) __builtin_amdgcn_raw_buffer_store_b128(v, orsrc, (c * plane + idx) * 4, 0, 2);
        }
        if (load) __syncthreads();
        if (!persistent) break;
    }
}

extern "C" int probe_launch(int mode, const void* src, void* out, int n_items, int rows, int src_item_bytes,
                            int src_tile_bytes, int grid, int work, const void* desc, void* stream)
{
    const int tiles = n_items * ((H + rows - 1) / rows);
    dim3      g(mode == 1 || mode == 3 ? grid : tiles);
    auto      s = (hipStream_t)stream;
#define L(M) hipLaunchKernelGGL(probe<M>, g, dim3(256), 0, s, (const uint8_t*)src, (float*)out, n_items, rows, \
                                src_item_bytes, src_tile_bytes, grid, work, (const uint64_t*)desc)
    switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    case 3: L(3); break;
    case 4: L(4); break;
    case 5: L(5); break;
    default: L(6); break;
    }
    return (int)hipGetLastError();
}

// Unaligned buffer loads: lane i reads 16 bytes at byte offset i (returns the bytes as loaded).
__global__ void probe_unaligned_k(const uint8_t* src, uint32_t* out, int n_bytes)
{
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, n_bytes, 0x00020000);
    const int  i  = threadIdx.x;
    u32x4      v  = __builtin_amdgcn_raw_buffer_load_b128(rs, i, 0, 0);
    out[i * 4 + 0] = v.x, out[i * 4 + 1] = v.y, out[i * 4 + 2] = v.z, out[i * 4 + 3] = v.w;
}

extern "C" int probe_unaligned(const void* src, void* out, int n_bytes, void* stream)
{
    hipLaunchKernelGGL(probe_unaligned_k, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t*)src,
                       (uint32_t*)out, n_bytes);
    return (int)hipGetLastError();
}
