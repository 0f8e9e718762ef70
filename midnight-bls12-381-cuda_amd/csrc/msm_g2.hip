// msm_g2.hip -- G2 instantiation of the MSM pipeline (msm_core.hpp) and its C entry points.
// Reference: bls12_381_g2_msm_cuda (icicle_curve_api.cu:695-705), msm_g2_cuda_impl (:454-618),
// G2 precompute (:620-650), own G2 registry (g2_registry.cu:72-82).
#include "msm_core.hpp"

using namespace mbls;
using G = Fq2;

extern "C" {

eIcicleError bls12_381_g2_msm_cuda(const mbls_fr_t* scalars, const mbls_g2_affine_t* bases, int msm_size,
                                   const MSMConfig* config, mbls_g2_projective_t* result) {
    return msm_call<G>(scalars, bases, msm_size, config, result, MSM_RAW);
}
eIcicleError bls12_381_icicle_g2_msm(const mbls_fr_t* scalars, const mbls_g2_affine_t* bases, int msm_size,
                                     const MSMConfig* config, mbls_g2_projective_t* results) {
    return msm_call<G>(scalars, bases, msm_size, config, results, MSM_ICICLE);
}
eIcicleError bls12_381_icicle_g2_msm_precompute_bases(const mbls_g2_affine_t* input_bases, int bases_size,
                                                      const MSMConfig* config, mbls_g2_affine_t* output_bases) {
    return precompute_call<G>(input_bases, bases_size, config, output_bases);
}
eIcicleError mbls_gen_g2_bases_range(mbls_g2_affine_t* out_device, uint64_t seed, size_t start, size_t n, void* stream) {
    if (!out_device) return MBLS_INVALID_POINTER;
    if (n == 0) return MBLS_SUCCESS;
    hipLaunchKernelGGL(k_gen_bases<G>, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, (hipStream_t)stream,
                       (uint8_t*)out_device, seed, start, n);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}
eIcicleError mbls_gen_g2_bases(mbls_g2_affine_t* out_device, uint64_t seed, size_t n, void* stream) {
    return mbls_gen_g2_bases_range(out_device, seed, 0, n, stream);
}
eIcicleError mbls_g2_msm_jacobian(const mbls_fr_t* scalars, const mbls_g2_affine_t* bases, int msm_size, const MSMConfig* config,
                                   mbls_g2_projective_t* results) {
    return msm_call<G>(scalars, bases, msm_size, config, results, MSM_JACOBIAN);
}
eIcicleError mbls_g2_sum_jacobian(const mbls_g2_projective_t* pts, int count, mbls_g2_projective_t* result,
                                  void* stream) {
    if (!pts || !result || count < 0) return MBLS_INVALID_ARGUMENT;
    hipLaunchKernelGGL(k_sum_jac<G>, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t*)pts, count,
                       (uint8_t*)result);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}
eIcicleError mbls_g2_jacobian_to_icicle(mbls_g2_projective_t* pts, int count, void* stream) {
    if (!pts || count < 0) return MBLS_INVALID_ARGUMENT;
    if (count == 0) return MBLS_SUCCESS;
    hipLaunchKernelGGL(k_jac_to_icicle<G>, dim3((count + 63) / 64), dim3(64), 0, (hipStream_t)stream, (const uint8_t*)pts, (uint8_t*)pts,
                       count);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

eIcicleError mbls_g2_msm_multi_device(const mbls_fr_t* scalars, const mbls_g2_affine_t* const* bases_per_dev, const int* devs,
                                      int ndev, int msm_size, const MSMConfig* config, mbls_g2_projective_t* result) {
    return msm_multi_device<G>(scalars, reinterpret_cast<const void* const*>(bases_per_dev), devs, ndev, msm_size, config,
                               result);
}

}  // extern "C"
