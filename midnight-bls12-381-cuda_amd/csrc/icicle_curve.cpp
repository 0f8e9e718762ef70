// icicle_curve.cpp -> lib/icicle/libicicle_backend_cuda_curve_bls12_381.so
//
// ICICLE curve backend (G1 / G2 MSM and base precomputation) over the HIP library: replaces
// the reference's icicle_curve_api.cu:243-665 registrations and its own G2 registry
// (g2_registry.cu:43-103; ICICLE core exports no G2 registration).  The impls forward to the
// ICICLE-semantics entry points (Montgomery flags honoured, (x, y, 1) standard projective
// result, batch computed), with the config bytes passed through unchanged.
#include <mutex>
#include <unordered_map>

#include "icicle_api.hpp"

namespace icicle {

// ---- G2 registry (function-local statics: no static-initialisation-order dependence) ----
namespace {
std::mutex& g2_mu() {
    static std::mutex m;
    return m;
}
std::unordered_map<std::string, MsmG2Impl>& g2_msm_map() {
    static std::unordered_map<std::string, MsmG2Impl> m;
    return m;
}
std::unordered_map<std::string, MsmG2PreComputeImpl>& g2_pre_map() {
    static std::unordered_map<std::string, MsmG2PreComputeImpl> m;
    return m;
}
}  // namespace

void register_g2_msm(const std::string& deviceType, MsmG2Impl impl) {
    std::lock_guard<std::mutex> lk(g2_mu());
    g2_msm_map()[deviceType] = std::move(impl);
}
void register_g2_msm_precompute_bases(const std::string& deviceType, MsmG2PreComputeImpl impl) {
    std::lock_guard<std::mutex> lk(g2_mu());
    g2_pre_map()[deviceType] = std::move(impl);
}
MsmG2Impl get_g2_msm_backend(const std::string& deviceType) {
    std::lock_guard<std::mutex> lk(g2_mu());
    auto it = g2_msm_map().find(deviceType);
    return it == g2_msm_map().end() ? MsmG2Impl() : it->second;
}
MsmG2PreComputeImpl get_g2_precompute_backend(const std::string& deviceType) {
    std::lock_guard<std::mutex> lk(g2_mu());
    auto it = g2_pre_map().find(deviceType);
    return it == g2_pre_map().end() ? MsmG2PreComputeImpl() : it->second;
}

}  // namespace icicle

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

const ::MSMConfig* c_cfg(const MSMConfig& c) { return reinterpret_cast<const ::MSMConfig*>(&c); }

eIcicleError msm_g1_impl(const Device&, const scalar_t* scalars, const affine_t* bases, int n, const MSMConfig& cfg,
                         projective_t* results) {
    return from_c(bls12_381_icicle_g1_msm(reinterpret_cast<const mbls_fr_t*>(scalars),
                                          reinterpret_cast<const mbls_g1_affine_t*>(bases), n, c_cfg(cfg),
                                          reinterpret_cast<mbls_g1_projective_t*>(results)));
}

eIcicleError msm_g1_precompute_impl(const Device&, const affine_t* in, int n, const MSMConfig& cfg, affine_t* out) {
    return from_c(bls12_381_icicle_g1_msm_precompute_bases(reinterpret_cast<const mbls_g1_affine_t*>(in), n, c_cfg(cfg),
                                                           reinterpret_cast<mbls_g1_affine_t*>(out)));
}

eIcicleError msm_g2_impl(const Device&, const scalar_t* scalars, const g2_affine_t* bases, int n, const MSMConfig& cfg,
                         g2_projective_t* results) {
    return from_c(bls12_381_icicle_g2_msm(reinterpret_cast<const mbls_fr_t*>(scalars),
                                          reinterpret_cast<const mbls_g2_affine_t*>(bases), n, c_cfg(cfg),
                                          reinterpret_cast<mbls_g2_projective_t*>(results)));
}

eIcicleError msm_g2_precompute_impl(const Device&, const g2_affine_t* in, int n, const MSMConfig& cfg,
                                    g2_affine_t* out) {
    return from_c(bls12_381_icicle_g2_msm_precompute_bases(reinterpret_cast<const mbls_g2_affine_t*>(in), n, c_cfg(cfg),
                                                           reinterpret_cast<mbls_g2_affine_t*>(out)));
}

// static registration under "CUDA" (icicle_curve_api.cu:660-665)
const bool registered = [] {
    const std::string dev = backend_device_type();
    if (register_msm_precompute_bases) register_msm_precompute_bases(dev, msm_g1_precompute_impl);
    if (register_msm) register_msm(dev, msm_g1_impl);
    register_g2_msm_precompute_bases(dev, msm_g2_precompute_impl);
    register_g2_msm(dev, msm_g2_impl);
    return true;
}();

}  // namespace

// C entry for tests / non-C++ hosts: invoke the registered G2 impl (what ICICLE's G2 frontend
// would do through get_g2_msm_backend)
extern "C" ::eIcicleError mbls_icicle_g2_msm_via_registry(const char* device_type, const mbls_fr_t* scalars,
                                                          const mbls_g2_affine_t* bases, int n, const ::MSMConfig* cfg,
                                                          mbls_g2_projective_t* results) {
    auto impl = icicle::get_g2_msm_backend(device_type ? device_type : "");
    if (!impl || !cfg) return MBLS_INVALID_ARGUMENT;
    const icicle::Device d = icicle::make_device(device_type, 0);
    return static_cast<::eIcicleError>(static_cast<int>(
        impl(d, reinterpret_cast<const icicle::scalar_t*>(scalars), reinterpret_cast<const icicle::g2_affine_t*>(bases), n,
             *reinterpret_cast<const icicle::MSMConfig*>(cfg), reinterpret_cast<icicle::g2_projective_t*>(results))));
}
