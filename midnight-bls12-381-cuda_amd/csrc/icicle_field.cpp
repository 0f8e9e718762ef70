// icicle_field.cpp -> lib/icicle/libicicle_backend_cuda_field_bls12_381.so
//
// ICICLE field backend (NTT + vector ops) for BLS12-381 Fr over the HIP library: replaces the
// reference's icicle_field_api.cu:97-352 registrations.  Each impl forwards to the C ABI with
// the same config bytes (icicle_api.hpp static_asserts the layouts).  Like the reference
// (icicle_field_api.cu:105), the Device argument is not read: ICICLE selects the device
// through the registered DeviceAPI (icicle_device.cpp) before dispatching.
#include <hip/hip_runtime_api.h>

#include <vector>

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

eIcicleError ntt_impl(const Device&, const scalar_t* input, int size, NTTDir dir, const NTTConfig<scalar_t>& config,
                      scalar_t* output) {
    return from_c(bls12_381_ntt_cuda(reinterpret_cast<const mbls_fr_t*>(input), size, static_cast<::NTTDir>(dir),
                                     reinterpret_cast<const ::NTTConfig*>(&config), reinterpret_cast<mbls_fr_t*>(output)));
}

eIcicleError ntt_init_domain_impl(const Device&, const scalar_t& root, const NTTInitDomainConfig& config) {
    return from_c(bls12_381_ntt_init_domain_cuda(reinterpret_cast<const mbls_fr_t*>(&root),
                                                 reinterpret_cast<const ::NTTInitDomainConfig*>(&config)));
}

eIcicleError ntt_release_domain_impl(const Device&, const scalar_t&) {
    return from_c(bls12_381_ntt_release_domain_cuda());
}

eIcicleError ntt_rou_impl(const Device&, uint64_t logn, scalar_t* rou) {
    return from_c(bls12_381_ntt_get_rou_from_domain(logn, reinterpret_cast<mbls_fr_t*>(rou)));
}

using BinOp = ::eIcicleError (*)(const mbls_fr_t*, const mbls_fr_t*, size_t, const ::VecOpsConfig*, mbls_fr_t*);

template <BinOp OP>
eIcicleError vec_impl(const Device&, const scalar_t* a, const scalar_t* b, uint64_t size, const VecOpsConfig& config,
                      scalar_t* out) {
    return from_c(OP(reinterpret_cast<const mbls_fr_t*>(a), reinterpret_cast<const mbls_fr_t*>(b), (size_t)size,
                     reinterpret_cast<const ::VecOpsConfig*>(&config), reinterpret_cast<mbls_fr_t*>(out)));
}

// ICICLE vector_sum: one sum per batch member (row-major batches); host operands are staged in
// the library's pooled scratch (bls12_381_vector_sum), no per-call hipMalloc
eIcicleError vec_sum_impl(const Device&, const scalar_t* a, uint64_t size, const VecOpsConfig& config, scalar_t* out) {
    if (!a || !out) return eIcicleError::INVALID_POINTER;
    if (size > (uint64_t)0x7fffffff) return eIcicleError::INVALID_ARGUMENT;
    return from_c(bls12_381_vector_sum(reinterpret_cast<const mbls_fr_t*>(a), (size_t)size,
                                       reinterpret_cast<const ::VecOpsConfig*>(&config), reinterpret_cast<mbls_fr_t*>(out)));
}

// static registration under "CUDA" (icicle_field_api.cu:344-352 registers the same set,
// minus vector_sum / get_rou_from_domain, which the HIP library also provides)
const bool registered = [] {
    const std::string dev = backend_device_type();
    if (register_ntt) register_ntt(dev, ntt_impl);
    if (register_ntt_init_domain) register_ntt_init_domain(dev, ntt_init_domain_impl);
    if (register_ntt_release_domain) register_ntt_release_domain(dev, ntt_release_domain_impl);
    if (register_ntt_get_rou_from_domain) register_ntt_get_rou_from_domain(dev, ntt_rou_impl);
    if (register_vector_add) register_vector_add(dev, vec_impl<bls12_381_vector_add>);
    if (register_vector_sub) register_vector_sub(dev, vec_impl<bls12_381_vector_sub>);
    if (register_vector_mul) register_vector_mul(dev, vec_impl<bls12_381_vector_mul>);
    if (register_scalar_mul_vec) register_scalar_mul_vec(dev, vec_impl<bls12_381_scalar_mul_vec>);
    if (register_scalar_add_vec) register_scalar_add_vec(dev, vec_impl<bls12_381_scalar_add_vec>);
    if (register_vector_sum) register_vector_sum(dev, vec_sum_impl);
    return true;
}();

}  // namespace
