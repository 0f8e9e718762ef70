// icicle_api.hpp -- ICICLE v4 backend-registration surface, declared so that the symbols our
// backend libraries reference mangle exactly like ICICLE core's.
//
// An unchanged midnight-zk reaches a GPU backend only through ICICLE: ICICLE core dlopens
// every backend library under ICICLE_BACKEND_INSTALL_DIR, whose static initialisers call
// icicle::register_*("CUDA", impl).  The Rust side hard-codes the device type "CUDA"
// (core/msm.rs:284, core/ntt.rs:351, core/vecops.rs:162), so the HIP backend registers under
// that name.  Declarations follow the reference's icicle_backend_api.cuh:69-226 and
// icicle_types.cuh:35-203 (type names, namespaces, parameter order) -- the reference's own
// claim about ICICLE's ABI; ICICLE's headers are not in this image, so the mangled names are
// checked against those declarations (tests/test_icicle_backend.py), not against ICICLE.
//
// Layout: every config struct is static_assert-ed against the C ABI struct of
// include/bls12_381_mi355x.h, and the impls reinterpret the pointers -- no copies.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <functional>
#include <memory>
#include <string>

#include "bls12_381_mi355x.h"

// ---- ICICLE's field / point templates (icicle_backend_api.cuh:69-83) -------------------
namespace bls12_381 {
struct fp_config;  // scalar field Fr
struct fq_config;  // base field Fq
struct G1;
struct G2;
}  // namespace bls12_381

template <typename Config>
class Field;
template <typename BaseField>
class Affine;
template <typename BaseField, typename ScalarField, typename Gen>
class Projective;
template <typename BaseConfig, typename BaseField>
class ComplexExtensionField;

// storage-only definitions with the blst / reference byte layouts (sizes checked below)
template <>
class Field<bls12_381::fp_config> {
   public:
    uint64_t limbs[4];
};
template <>
class Field<bls12_381::fq_config> {
   public:
    uint64_t limbs[6];
};
template <>
class ComplexExtensionField<bls12_381::fq_config, Field<bls12_381::fq_config>> {
   public:
    Field<bls12_381::fq_config> c0, c1;
};
template <typename BaseField>
class Affine {
   public:
    BaseField x, y;
};
template <typename BaseField, typename ScalarField, typename Gen>
class Projective {
   public:
    BaseField x, y, z;
};

namespace icicle {

using scalar_t = Field<bls12_381::fp_config>;
using point_field_t = Field<bls12_381::fq_config>;
using affine_t = Affine<point_field_t>;
using projective_t = Projective<point_field_t, scalar_t, bls12_381::G1>;
using g2_field_t = ComplexExtensionField<bls12_381::fq_config, point_field_t>;
using g2_affine_t = Affine<g2_field_t>;
using g2_projective_t = Projective<g2_field_t, scalar_t, bls12_381::G2>;

// ---- runtime types (icicle_types.cuh:47-201; error numbering of ICICLE errors.h) --------
enum class eIcicleError {
    SUCCESS = 0,
    INVALID_DEVICE = 1,
    OUT_OF_MEMORY = 2,
    INVALID_POINTER = 3,
    ALLOCATION_FAILED = 4,
    DEALLOCATION_FAILED = 5,
    COPY_FAILED = 6,
    SYNCHRONIZATION_FAILED = 7,
    STREAM_CREATION_FAILED = 8,
    STREAM_DESTRUCTION_FAILED = 9,
    API_NOT_IMPLEMENTED = 10,
    INVALID_ARGUMENT = 11,
    BACKEND_LOAD_FAILED = 12,
    LICENSE_CHECK_ERROR = 13,
    UNKNOWN_ERROR = 14
};

// ICICLE's device descriptor (vendored include/icicle/device.h:55-57): the type string is an
// inline char[32], so `id` sits at byte offset 32 (the reference's icicle_types.cuh:69-72
// declares {const char*, int}, which reads `id` from inside the string)
struct Device {
    char type[32];
    int id;
};
static_assert(offsetof(Device, id) == 32 && sizeof(Device) == 36, "icicle::Device layout (device.h:55-57)");
// what ICICLE's Device(const char*, int) constructor produces (zero-padded, truncated type)
inline Device make_device(const char* type, int id) {
    Device d;
    for (size_t i = 0; i < sizeof d.type; ++i) d.type[i] = 0;
    for (size_t i = 0; type && type[i] && i + 1 < sizeof d.type; ++i) d.type[i] = type[i];
    d.id = id;
    return d;
}

typedef void* icicleStreamHandle;

enum class NTTDir { kForward = 0, kInverse = 1 };
enum class Ordering { kNN = 0, kNR = 1, kRN = 2, kRR = 3, kNM = 4, kMN = 5 };

template <typename S>
struct NTTConfig {
    icicleStreamHandle stream;
    S coset_gen;
    int batch_size;
    bool columns_batch;
    Ordering ordering;
    bool are_inputs_on_device;
    bool are_outputs_on_device;
    bool is_async;
    void* ext;
};

struct NTTInitDomainConfig {
    icicleStreamHandle stream;
    bool is_async;
    void* ext;
};

struct MSMConfig {
    icicleStreamHandle stream;
    int precompute_factor;
    int c;
    int bitsize;
    int batch_size;
    bool are_points_shared_in_batch;
    bool are_scalars_on_device;
    bool are_scalars_montgomery_form;
    bool are_points_on_device;
    bool are_points_montgomery_form;
    bool are_results_on_device;
    bool is_async;
    void* ext;
};

struct VecOpsConfig {  // ICICLE v4 layout
    icicleStreamHandle stream;
    bool is_a_on_device;
    bool is_b_on_device;
    bool is_result_on_device;
    bool is_async;
    int batch_size;
    bool columns_batch;
    void* ext;
};

// ---- impl signatures (icicle_backend_api.cuh:118-219) ----------------------------------
using NttImpl = std::function<eIcicleError(const Device& device, const scalar_t* input, int size, NTTDir dir,
                                           const NTTConfig<scalar_t>& config, scalar_t* output)>;
using NttInitDomainImpl =
    std::function<eIcicleError(const Device& device, const scalar_t& primitive_root, const NTTInitDomainConfig& config)>;
using NttReleaseDomainImpl = std::function<eIcicleError(const Device& device, const scalar_t& phantom)>;
using NttGetRouFromDomainImpl = std::function<eIcicleError(const Device& device, uint64_t logn, scalar_t* rou)>;
using scalarVectorOpImpl = std::function<eIcicleError(const Device& device, const scalar_t* scalar_a,
                                                      const scalar_t* vec_b, uint64_t size,
                                                      const VecOpsConfig& config, scalar_t* output)>;
using VectorReduceOpImpl = std::function<eIcicleError(const Device& device, const scalar_t* vec_a, uint64_t size,
                                                      const VecOpsConfig& config, scalar_t* output)>;
using MsmImpl = std::function<eIcicleError(const Device& device, const scalar_t* scalars, const affine_t* bases,
                                           int msm_size, const MSMConfig& config, projective_t* results)>;
using MsmPreComputeImpl = std::function<eIcicleError(const Device& device, const affine_t* input_bases,
                                                     int bases_size, const MSMConfig& config, affine_t* output_bases)>;
using MsmG2Impl = std::function<eIcicleError(const Device& device, const scalar_t* scalars, const g2_affine_t* bases,
                                             int msm_size, const MSMConfig& config, g2_projective_t* results)>;
using MsmG2PreComputeImpl =
    std::function<eIcicleError(const Device& device, const g2_affine_t* input_bases, int bases_size,
                               const MSMConfig& config, g2_affine_t* output_bases)>;

// ---- registration entry points, resolved from ICICLE core at dlopen time (weak: the
//      libraries also load standalone, e.g. in tests, where the calls are skipped) ----------
__attribute__((weak)) void register_ntt(const std::string& deviceType, NttImpl impl);
__attribute__((weak)) void register_ntt_init_domain(const std::string& deviceType, NttInitDomainImpl impl);
__attribute__((weak)) void register_ntt_release_domain(const std::string& deviceType, NttReleaseDomainImpl impl);
__attribute__((weak)) void register_ntt_get_rou_from_domain(const std::string& deviceType, NttGetRouFromDomainImpl impl);
__attribute__((weak)) void register_vector_add(const std::string& deviceType, scalarVectorOpImpl impl);
__attribute__((weak)) void register_vector_sub(const std::string& deviceType, scalarVectorOpImpl impl);
__attribute__((weak)) void register_vector_mul(const std::string& deviceType, scalarVectorOpImpl impl);
__attribute__((weak)) void register_scalar_mul_vec(const std::string& deviceType, scalarVectorOpImpl impl);
__attribute__((weak)) void register_scalar_add_vec(const std::string& deviceType, scalarVectorOpImpl impl);
__attribute__((weak)) void register_vector_sum(const std::string& deviceType, VectorReduceOpImpl impl);
__attribute__((weak)) void register_msm(const std::string& deviceType, MsmImpl impl);
__attribute__((weak)) void register_msm_precompute_bases(const std::string& deviceType, MsmPreComputeImpl impl);
// G2: ICICLE core does not export these (G2_ENABLED builds only); the curve backend defines
// them itself, like the reference's g2_registry.cu:72-101
void register_g2_msm(const std::string& deviceType, MsmG2Impl impl);
void register_g2_msm_precompute_bases(const std::string& deviceType, MsmG2PreComputeImpl impl);
MsmG2Impl get_g2_msm_backend(const std::string& deviceType);
MsmG2PreComputeImpl get_g2_precompute_backend(const std::string& deviceType);

// ---- device API (vtable order of the vendored include/icicle/device_api.h:52-131, which the
//      reference's cuda_device_api.cu:38-149 overrides) ----
// device_api.h:44 (plain enum there; same int values)
enum class eCopyDirection { HostToDevice = 0, DeviceToHost = 1, DeviceToDevice = 2, HostToHost = 3 };
struct DeviceProperties {
    bool using_host_memory;
    int num_memory_regions;
    bool supports_pinned_memory;
};
class DeviceAPI {
   public:
    virtual ~DeviceAPI() {}
    virtual eIcicleError set_device(const Device& device) = 0;
    virtual eIcicleError get_device_count(int& device_count) const = 0;
    virtual eIcicleError allocate_memory(void** ptr, size_t size) const = 0;
    virtual eIcicleError allocate_memory_async(void** ptr, size_t size, icicleStreamHandle stream) const = 0;
    virtual eIcicleError free_memory(void* ptr) const = 0;
    virtual eIcicleError free_memory_async(void* ptr, icicleStreamHandle stream) const = 0;
    virtual eIcicleError get_available_memory(size_t& total, size_t& free) const = 0;
    virtual eIcicleError memset(void* ptr, int value, size_t size) const = 0;
    virtual eIcicleError memset_async(void* ptr, int value, size_t size, icicleStreamHandle stream) const = 0;
    virtual eIcicleError copy(void* dst, const void* src, size_t size, eCopyDirection direction) const = 0;
    virtual eIcicleError copy_async(void* dst, const void* src, size_t size, eCopyDirection direction,
                                    icicleStreamHandle stream) const = 0;
    virtual eIcicleError synchronize(icicleStreamHandle stream = nullptr) const = 0;
    virtual eIcicleError create_stream(icicleStreamHandle* stream) const = 0;
    virtual eIcicleError destroy_stream(icicleStreamHandle stream) const = 0;
    virtual eIcicleError get_device_properties(DeviceProperties& properties) const = 0;
};
__attribute__((weak)) void register_deviceAPI(const std::string& deviceType, std::shared_ptr<DeviceAPI> api);

// the device type string the Rust side selects (see header comment)
inline const char* backend_device_type() { return "CUDA"; }

// ---- byte-compatibility with the C ABI --------------------------------------------------
static_assert(sizeof(scalar_t) == sizeof(mbls_fr_t), "Fr layout");
static_assert(sizeof(affine_t) == sizeof(mbls_g1_affine_t), "G1 affine layout");
static_assert(sizeof(projective_t) == sizeof(mbls_g1_projective_t), "G1 projective layout");
static_assert(sizeof(g2_affine_t) == sizeof(mbls_g2_affine_t), "G2 affine layout");
static_assert(sizeof(g2_projective_t) == sizeof(mbls_g2_projective_t), "G2 projective layout");
static_assert(sizeof(MSMConfig) == sizeof(::MSMConfig) && offsetof(MSMConfig, is_async) == offsetof(::MSMConfig, is_async) &&
                  offsetof(MSMConfig, ext) == offsetof(::MSMConfig, ext),
              "MSMConfig layout");
static_assert(sizeof(NTTConfig<scalar_t>) == sizeof(::NTTConfig) &&
                  offsetof(NTTConfig<scalar_t>, ordering) == offsetof(::NTTConfig, ordering) &&
                  offsetof(NTTConfig<scalar_t>, ext) == offsetof(::NTTConfig, ext),
              "NTTConfig layout");
static_assert(sizeof(NTTInitDomainConfig) == sizeof(::NTTInitDomainConfig), "NTTInitDomainConfig layout");
static_assert(sizeof(VecOpsConfig) == sizeof(::VecOpsConfig) && offsetof(VecOpsConfig, batch_size) == offsetof(::VecOpsConfig, batch_size) &&
                  offsetof(VecOpsConfig, ext) == offsetof(::VecOpsConfig, ext),
              "VecOpsConfig layout");

inline eIcicleError from_c(::eIcicleError e) { return static_cast<eIcicleError>(static_cast<int>(e)); }

}  // namespace icicle
