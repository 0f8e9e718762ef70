// icicle_device.cpp -> lib/icicle/libicicle_backend_cuda_device.so
//
// ICICLE DeviceAPI for the "CUDA" device type implemented on HIP (replaces the reference's
// cuda_device_api.cu:38-149): ICICLE core routes memory, copies, streams and device
// selection for the device type through this object, so an unchanged midnight-zk gets HIP
// memory / hipStream_t handles, which the field and curve backends then consume.
// Error mapping follows the reference's choices (ALLOCATION_FAILED for malloc, COPY_FAILED for
// copies, ...).  Async allocation uses hipMallocAsync (stream-ordered pool).
#include <hip/hip_runtime_api.h>

#include "icicle_api.hpp"

namespace {
using icicle::eIcicleError;
using icicle::Device;
using icicle::scalar_t;
using icicle::affine_t;
using icicle::projective_t;
using icicle::g2_affine_t;
using icicle::g2_projective_t;
using icicle::NTTDir;
using icicle::NTTConfig;
using icicle::NTTInitDomainConfig;
using icicle::MSMConfig;
using icicle::VecOpsConfig;
using icicle::from_c;
using icicle::backend_device_type;
using namespace icicle;  // register_* (no clashes: the C ABI has no such names)

hipMemcpyKind kind(eCopyDirection d) {
    switch (d) {
        case eCopyDirection::HostToDevice: return hipMemcpyHostToDevice;
        case eCopyDirection::DeviceToHost: return hipMemcpyDeviceToHost;
        case eCopyDirection::HostToHost: return hipMemcpyHostToHost;
        default: return hipMemcpyDeviceToDevice;
    }
}
hipStream_t hs(icicleStreamHandle s) { return static_cast<hipStream_t>(s); }
eIcicleError ok_or(hipError_t e, eIcicleError fail) { return e == hipSuccess ? eIcicleError::SUCCESS : fail; }

class HipDeviceAPI final : public DeviceAPI {
   public:
    eIcicleError set_device(const Device& device) override {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || device.id < 0 || device.id >= count)
            return eIcicleError::INVALID_DEVICE;
        return ok_or(hipSetDevice(device.id), eIcicleError::INVALID_DEVICE);
    }
    eIcicleError get_device_count(int& device_count) const override {
        return ok_or(hipGetDeviceCount(&device_count), eIcicleError::INVALID_DEVICE);
    }
    eIcicleError allocate_memory(void** ptr, size_t size) const override {
        return ok_or(hipMalloc(ptr, size), eIcicleError::ALLOCATION_FAILED);
    }
    eIcicleError allocate_memory_async(void** ptr, size_t size, icicleStreamHandle stream) const override {
        return ok_or(hipMallocAsync(ptr, size, hs(stream)), eIcicleError::ALLOCATION_FAILED);
    }
    eIcicleError free_memory(void* ptr) const override {
        return ok_or(hipFree(ptr), eIcicleError::DEALLOCATION_FAILED);
    }
    eIcicleError free_memory_async(void* ptr, icicleStreamHandle stream) const override {
        return ok_or(hipFreeAsync(ptr, hs(stream)), eIcicleError::DEALLOCATION_FAILED);
    }
    eIcicleError get_available_memory(size_t& total, size_t& free) const override {
        return ok_or(hipMemGetInfo(&free, &total), eIcicleError::UNKNOWN_ERROR);
    }
    eIcicleError memset(void* ptr, int value, size_t size) const override {
        return ok_or(hipMemset(ptr, value, size), eIcicleError::UNKNOWN_ERROR);
    }
    eIcicleError memset_async(void* ptr, int value, size_t size, icicleStreamHandle stream) const override {
        return ok_or(hipMemsetAsync(ptr, value, size, hs(stream)), eIcicleError::UNKNOWN_ERROR);
    }
    eIcicleError copy(void* dst, const void* src, size_t size, eCopyDirection direction) const override {
        return ok_or(hipMemcpy(dst, src, size, kind(direction)), eIcicleError::COPY_FAILED);
    }
    eIcicleError copy_async(void* dst, const void* src, size_t size, eCopyDirection direction,
                            icicleStreamHandle stream) const override {
        return ok_or(hipMemcpyAsync(dst, src, size, kind(direction), hs(stream)), eIcicleError::COPY_FAILED);
    }
    eIcicleError synchronize(icicleStreamHandle stream = nullptr) const override {
        return ok_or(stream ? hipStreamSynchronize(hs(stream)) : hipDeviceSynchronize(),
                     eIcicleError::SYNCHRONIZATION_FAILED);
    }
    eIcicleError create_stream(icicleStreamHandle* stream) const override {
        hipStream_t s = nullptr;
        const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        *stream = static_cast<icicleStreamHandle>(s);
        return ok_or(e, eIcicleError::STREAM_CREATION_FAILED);
    }
    eIcicleError destroy_stream(icicleStreamHandle stream) const override {
        // the library forgets the handle first (its scratch contexts are pooled per device, not
        // per stream: nothing is freed or leaked here, and a recycled handle value is not taken
        // to be ordered after this stream's work)
        (void)mbls_release_stream(stream);
        return ok_or(hipStreamDestroy(hs(stream)), eIcicleError::STREAM_DESTRUCTION_FAILED);
    }
    eIcicleError get_device_properties(DeviceProperties& properties) const override {
        properties.using_host_memory = false;
        properties.num_memory_regions = 1;
        properties.supports_pinned_memory = true;
        return eIcicleError::SUCCESS;
    }
};

const bool registered = [] {
    if (register_deviceAPI) register_deviceAPI(backend_device_type(), std::make_shared<HipDeviceAPI>());
    return true;
}();

}  // namespace
