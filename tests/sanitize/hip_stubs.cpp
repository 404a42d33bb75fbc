// hip_stubs.cpp -- a device-free stand-in for the HIP runtime and the device half of the C ABI, so the
// host layer (aeon_amd/csrc/host.cpp: decoder configuration, thread_pool, window draws) links into a
// sanitizer build without libamdhip64 (tests/sanitize/host_driver.cpp, Makefile targets `sanitize` /
// `tsan`).  Every device entry point fails with "no device": a decode window's flush cannot run here,
// which is the point -- the driver exercises only the host phases.  Host-only entry points the layer
// calls (PNG / JPEG headers, PNG decode) forward to the real implementations.
#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdlib>
#include <string>

#include "../../aeon_amd/csrc/host.hpp"
#include "../../aeon_amd/csrc/jpeg.hpp"

namespace aeon_hip {
void jpeg_info(const void* data, size_t size, int* w, int* h, int* ncomp);
void png_header(const void* data, size_t size, int* w, int* h, int* depth, int* ctype);
void png_decode(const void* data, size_t size, int mode, void* dst, size_t stride, int* out_elem_bytes);
void ctx_share_pool(aeon_hip_ctx*, thread_pool*) {}
} // namespace aeon_hip

namespace {
thread_local std::string g_err;
int no_device()
{
    g_err = "sanitizer build: no device";
    return AEON_HIP_EDEVICE;
}
template <typename F>
int host_call(F&& f)
{
    try {
        f();
        return 0;
    } catch (const aeon_hip::jpeg_error& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return AEON_HIP_EINVAL;
    }
}
} // namespace

extern "C" {
// ---- HIP runtime ----
// host memory and event / stream handles work (the stager's staging runs on them); device memory,
// copies and launches do not
hipError_t hipMalloc(void**, size_t) { return hipErrorNoDevice; }
hipError_t hipHostMalloc(void** p, size_t n, unsigned int)
{
    *p = std::malloc(n ? n : 1);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void*) { return hipSuccess; }
hipError_t hipHostFree(void* p)
{
    std::free(p);
    return hipSuccess;
}
hipError_t hipGetDevice(int* d)
{
    *d = 0;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipHostRegister(void*, size_t, unsigned int) { return hipErrorNoDevice; }
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipErrorNoDevice; }
hipError_t hipEventDestroy(hipEvent_t e)
{
    delete reinterpret_cast<int*>(e);
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e)
{
    *e = reinterpret_cast<hipEvent_t>(new int(0));
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipErrorNoDevice; }
hipError_t hipStreamCreate(hipStream_t* s)
{
    *s = reinterpret_cast<hipStream_t>(new int(0));
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) { return hipStreamCreate(s); }
hipError_t hipStreamDestroy(hipStream_t s)
{
    delete reinterpret_cast<int*>(s);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void*, const void*, size_t, hipMemcpyKind, hipStream_t) { return hipErrorNoDevice; }
hipError_t hipMemcpy(void*, const void*, size_t, hipMemcpyKind) { return hipErrorNoDevice; }
hipError_t hipPointerGetAttributes(hipPointerAttribute_t*, const void*) { return hipErrorInvalidValue; }
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t) { return "no device (sanitizer build)"; }
int         roctxRangePushA(const char*) { return 0; }
int         roctxRangePop() { return 0; }

// ---- the device half of include/aeon_hip.h ----
int aeon_hip_ctx_create(int, aeon_hip_ctx**) { return no_device(); }
int aeon_hip_ctx_destroy(aeon_hip_ctx*) { return 0; }
int aeon_hip_augment_batch(aeon_hip_ctx*, int, const aeon_img_desc*, const void*, const aeon_aug_params*,
                           const aeon_out_desc*, void*, void*)
{
    return no_device();
}
int aeon_hip_mask_batch(aeon_hip_ctx*, int, const aeon_img_desc*, const void*, const aeon_aug_params*,
                        const aeon_out_desc*, void*, void*)
{
    return no_device();
}
int aeon_hip_augment_pair_batch(aeon_hip_ctx*, int, const aeon_img_desc*, const void*, const aeon_img_desc*, const void*,
                                const aeon_aug_params*, const aeon_out_desc*, void*, const aeon_out_desc*, void*, void*)
{
    return no_device();
}
int aeon_hip_transpose_batch(aeon_hip_ctx*, const void*, void*, int64_t, int64_t, int, void*) { return no_device(); }
int aeon_hip_decode_jpeg_batch(aeon_hip_ctx*, int, const void* const*, const size_t*, const aeon_img_desc*, void*,
                               void*)
{
    return no_device();
}
int aeon_hip_synchronize(aeon_hip_ctx*, void*) { return no_device(); }
int aeon_hip_release_stream(aeon_hip_ctx*, void*) { return no_device(); }
const char* aeon_hip_last_error(void) { return g_err.c_str(); }

// ---- host-only entry points: the real implementations ----
int aeon_jpeg_info(const void* data, size_t size, int* w, int* h, int* n)
{
    return host_call([&] { aeon_hip::jpeg_info(data, size, w, h, n); });
}
int aeon_png_info(const void* data, size_t size, int* w, int* h, int* depth, int* ctype)
{
    return host_call([&] { aeon_hip::png_header(data, size, w, h, depth, ctype); });
}
int aeon_decode_png(const void* data, size_t size, int mode, void* dst, size_t stride, int* eb)
{
    return host_call([&] { aeon_hip::png_decode(data, size, mode, dst, stride, eb); });
}
} // extern "C"
