// batch_transpose.hip -- aeon's batch_major=false layout on the GPU.
//
// aeon copies every decoded batch into the caller's buffer transposed when the loader runs
// with batch_major=false (batch_iterator_fbm::filler, src/batch_iterator.cpp:125-136 ->
// fixed_buffer_map::copy(..., transpose=true), src/buffer_batch.cpp:251-280 -> transpose_buf /
// transpose_regular, src/buffer_batch.cpp:186-244):  dst[c * rows + r] = src[r * cols + c] for
// a rows x cols matrix of element_size-byte elements (rows = batch size, cols = elements per
// item).  Pure data movement: HBM-bound, read once + written once through a 64 x 64 LDS tile so
// both the reads (along c) and the writes (along r) are coalesced.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aeon_hip {

constexpr int kTile = 64;

template <typename T>
__global__ __launch_bounds__(256) void transpose_tiles(const T* __restrict__ src, T* __restrict__ dst, int64_t rows,
                                                      int64_t cols)
{
    __shared__ T tile[kTile][kTile + 1]; // +1: the column-wise reads hit distinct banks
    const int64_t c0 = (int64_t)blockIdx.x * kTile, r0 = (int64_t)blockIdx.y * kTile;
    const int     tx = threadIdx.x & (kTile - 1), ty = threadIdx.x / kTile; // 64 x 4 lanes
#pragma unroll 4
    for (int j = ty; j < kTile; j += 256 / kTile) {
        const int64_t r = r0 + j, c = c0 + tx;
        if (r < rows && c < cols) tile[j][tx] = src[r * cols + c];
    }
    __syncthreads();
#pragma unroll 4
    for (int j = ty; j < kTile; j += 256 / kTile) {
        const int64_t c = c0 + j, r = r0 + tx;
        if (c < cols && r < rows) dst[c * rows + r] = tile[tx][j];
    }
}

hipError_t launch_transpose(const void* src, void* dst, int64_t rows, int64_t cols, int element_size,
                            hipStream_t stream)
{
    const dim3 grid((unsigned)((cols + kTile - 1) / kTile), (unsigned)((rows + kTile - 1) / kTile)), block(256);
    switch (element_size) {
    case 1: hipLaunchKernelGGL(transpose_tiles<uint8_t>, grid, block, 0, stream, (const uint8_t*)src, (uint8_t*)dst, rows, cols); break;
    case 2: hipLaunchKernelGGL(transpose_tiles<uint16_t>, grid, block, 0, stream, (const uint16_t*)src, (uint16_t*)dst, rows, cols); break;
    case 4: hipLaunchKernelGGL(transpose_tiles<uint32_t>, grid, block, 0, stream, (const uint32_t*)src, (uint32_t*)dst, rows, cols); break;
    case 8: hipLaunchKernelGGL(transpose_tiles<uint64_t>, grid, block, 0, stream, (const uint64_t*)src, (uint64_t*)dst, rows, cols); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// Job-table upload as a kernel on the launch stream (AEON_HIP_JOBS=3): the slot's pinned host
// table is read over PCIe with system-coherent 16-byte loads (no L2 copy of an older use of the
// slot can be returned) and written to the slot's device table.  Kernel-to-kernel ordering on one
// queue then replaces the cross-queue wait on an SDMA copy.
__global__ __launch_bounds__(256) void upload_table(const void* host_src, uint4* __restrict__ dst, int n16)
{
    const auto src = __builtin_amdgcn_make_buffer_rsrc((void*)host_src, (short)0, n16 * 16, 0x00020000);
    const int  i   = blockIdx.x * 256 + threadIdx.x;
    if (i < n16) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(src, i * 16, 0, 1 | 16); // sc0 sc1
        dst[i]       = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

hipError_t launch_upload_table(const void* host_dev, void* dst, size_t bytes, hipStream_t stream)
{
    const int n16 = (int)((bytes + 15) / 16);
    hipLaunchKernelGGL(upload_table, dim3((n16 + 255) / 256), dim3(256), 0, stream, host_dev, (uint4*)dst, n16);
    return hipGetLastError();
}

} // namespace aeon_hip
