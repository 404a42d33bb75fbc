// plan_kernels.hip -- the device planner: per-record jobs built on the GPU from the caller's
// descriptors + params (stage.cpp run_direct), replacing both the host's per-record planning and
// the job-table upload.  One lane per record: eight system-coherent 16-byte loads of its
// PlanRecord from the pinned slot (PCIe), plan_direct (plan_record.hpp -- the host planner's own
// code), one 256-byte AugJob store into the slot's device table.  The tile kernel that follows on
// the same stream reads the table through scalar loads.
#include <hip/hip_runtime.h>

#include "plan_record.hpp"

namespace aeon_hip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void plan_records(const PlanRecord* host_records, AugJob* __restrict__ jobs,
                                                   PlanArgs a)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= a.n) return;
    // sc0 sc1: read through to host memory (the slot was written by the host since its last use)
    const auto  src = __builtin_amdgcn_make_buffer_rsrc((void*)host_records, (short)0, a.n * (int)sizeof(PlanRecord),
                                                        0x00020000);
    u32x4       w[8];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = __builtin_amdgcn_raw_buffer_load_b128(src, i * 128 + k * 16, 0, 1 | 16);
    PlanRecord R;
    __builtin_memcpy(&R, w, sizeof(R));
    AugJob J;
    plan_direct(R.desc, a.src_base, R.params, a.out, a.out_base + (uint64_t)i * a.item_stride, a.is_mask != 0, J);
    J.tiles = (J.win_h + a.rows_per_tile - 1) / a.rows_per_tile;
    jobs[i] = J;
}

hipError_t launch_plan_records(const void* host_records, void* jobs, const PlanArgs& a, hipStream_t stream)
{
    hipLaunchKernelGGL(plan_records, dim3((a.n + 63) / 64), dim3(64), 0, stream, (const PlanRecord*)host_records,
                       (AugJob*)jobs, a);
    return hipGetLastError();
}

} // namespace aeon_hip
