// plan_kernels.hip -- the device planner: per-record jobs built on the GPU from the caller's
// descriptors + params (stage.cpp run_direct), replacing both the host's per-record planning and
// the job-table upload: the records' PlanRecords come from the pinned slot over PCIe, each is
// planned by plan_direct (plan_record.hpp -- the host planner's own code) and its AugJob lands in
// the slot's device table, which the tile kernel that follows on the same stream reads through
// scalar loads.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "plan_record.hpp"

namespace aeon_hip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A workgroup plans PER records: its lanes bring the records' 16-byte pieces over PCIe (many lanes
// and workgroups keep many reads in flight: with one lane reading a whole record the kernel took
// 11.8 us for 256 records, against 5.2 us for a 64 KiB table upload); lanes 0..PER-1 plan one record
// each into LDS; all lanes store the jobs 16 bytes apiece.
template <int PER, int LANES>
__global__ __launch_bounds__(LANES) void plan_records(const PlanRecord* host_records, AugJob* __restrict__ jobs, PlanArgs a)
{
    __shared__ u32x4 recs[PER * kPlanRecordPieces];
    __shared__ u32x4 out[PER * 16];
    const int tid = threadIdx.x;
    const int r0  = blockIdx.x * PER;
    const int nr  = min(PER, a.n - r0);
    // sc0 sc1: read through to host memory (the slot was written by the host since its last use)
    const auto src = __builtin_amdgcn_make_buffer_rsrc((void*)host_records, (short)0, a.n * (int)sizeof(PlanRecord),
                                                       0x00020000);
    for (int i = tid; i < nr * kPlanRecordPieces; i += LANES)
        recs[i] = __builtin_amdgcn_raw_buffer_load_b128(src, r0 * (int)sizeof(PlanRecord) + i * 16, 0, 1 | 16);
    __syncthreads();
    if (tid < nr) {
        PlanRecord R;
        __builtin_memcpy(&R, &recs[tid * kPlanRecordPieces], sizeof(R));
        const int i = r0 + tid;
        AugJob    J;
        plan_direct(R.desc, a.src_base, R.params, a.out, a.out_base + (uint64_t)i * a.item_stride, a.is_mask != 0, J);
        J.tiles = (J.win_h + a.rows_per_tile - 1) / a.rows_per_tile;
        __builtin_memcpy(&out[tid * 16], &J, sizeof(J));
    }
    __syncthreads();
    u32x4* dst = (u32x4*)(jobs + r0);
    for (int k = tid; k < nr * 16; k += LANES) dst[k] = out[k];
}

hipError_t launch_plan_records(const void* host_records, void* jobs, const PlanArgs& a, hipStream_t stream)
{
    // 16 records per 128-lane workgroup (measured against 1, 4 and 8 per workgroup)
    hipLaunchKernelGGL((plan_records<16, 128>), dim3((a.n + 15) / 16), dim3(128), 0, stream,
                       (const PlanRecord*)host_records, (AugJob*)jobs, a);
    return hipGetLastError();
}

} // namespace aeon_hip
