// points.hip -- batch point-form conversions of the reference's C ABI (point_ops.cu:759,844,924):
//   bls12_381_g1_affine_to_projective  Montgomery affine -> Jacobian (x, y, 1); identity (0, 0) ->
//                                      (0, 1, 0)  (Projective::from_affine, point.cuh:477-482)
//   bls12_381_g1_projective_to_affine  Jacobian -> affine (X / Z^2, Y / Z^3); Z = 0 -> (0, 0)
//   bls12_381_g2_projective_to_affine  the same over Fq2        (Projective::to_affine, point.cuh:504-525)
// All values stay in Montgomery form (no standard-form conversion, as in the reference).
// Placement follows VecOpsConfig: is_a_on_device for the input, is_result_on_device for the
// output; host buffers are staged through the leased scratch context (common.cpp) instead of the
// reference's per-call cudaMalloc / cudaFree.
//
// projective_to_affine: one Montgomery batch inversion per thread over a run of K points
// (Montgomery's trick: prefix products of the Z's, one inversion, a backward sweep), so a point
// costs ~3 products plus 1/K of a binary-GCD inversion (mbls_binv.hpp, ~59 products) instead of
// the reference's one Fermat inversion per point (point_ops.cu:75-99).  The prefix products are
// kept in the output buffer (its x slot) between the two sweeps: registers hold one running
// product only.  Identity inputs (Z = 0) are skipped by the prefix chain.
#include <hip/hip_runtime.h>

#include "mbls_common.hpp"
#include "mbls_curve.hpp"

namespace mbls {

static constexpr int POINT_MAX_BATCH = 1 << 26;  // point_ops.cu:745 MAX_POINT_BATCH_SIZE
static constexpr int P2A_RUN = 8;                // points per thread sharing one inversion

template <class F>
struct PointBytes;
template <>
struct PointBytes<Fq> {
    static constexpr size_t AFF = 96, JAC = 144;
};
template <>
struct PointBytes<Fq2> {
    static constexpr size_t AFF = 192, JAC = 288;
};

template <class F>
__global__ void k_affine_to_jac(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int n) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const Affine<F> a = load_affine<F>(in, i);
    Jacobian<F> p;
    if (a.is_inf()) {
        p.x = F::zero();
        p.y = F::one();
        p.z = F::zero();
    } else {
        p.x = a.x;
        p.y = a.y;
        p.z = F::one();
    }
    store_jac<F>(out, i, p);
}

// thread t converts points [t K, t K + K); the prefix product before point i is parked in the
// x slot of out[i] (the affine x is written over it in the backward sweep)
template <class F>
__global__ __launch_bounds__(64) void k_jac_to_affine(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int n) {
    const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int i0 = t * P2A_RUN;
    if (i0 >= n) return;
    const int i1 = i0 + P2A_RUN < n ? i0 + P2A_RUN : n;
    constexpr size_t FB = FieldIO<F>::BYTES;
    F acc = F::one();
    for (int i = i0; i < i1; ++i) {
        const uint8_t* p = in + (size_t)i * 3 * FB;
        const F z = FieldIO<F>::ld(p + 2 * FB);
        FieldIO<F>::st(out + (size_t)i * 2 * FB, acc);  // prefix before i
        if (!z.is_zero()) acc = acc * z;
    }
    F inv_acc = inv(acc);  // 1 / prod of the non-zero Z's of the run
    for (int i = i1 - 1; i >= i0; --i) {
        const uint8_t* p = in + (size_t)i * 3 * FB;
        const F z = FieldIO<F>::ld(p + 2 * FB);
        uint8_t* o = out + (size_t)i * 2 * FB;
        if (z.is_zero()) {
            FieldIO<F>::st(o, F::zero());
            FieldIO<F>::st(o + FB, F::zero());
            continue;
        }
        const F prefix = FieldIO<F>::ld(o);
        const F zi = inv_acc * prefix;  // 1 / z
        inv_acc = inv_acc * z;          // 1 / (prefix product before i)
        const F zi2 = sqr(zi);
        const F x = FieldIO<F>::ld(p), y = FieldIO<F>::ld(p + FB);
        FieldIO<F>::st(o, x * zi2);
        FieldIO<F>::st(o + FB, y * zi2 * zi);
    }
}

// in == out (in place) is allowed for affine -> projective only when the buffers do not overlap
// partially; the reference does not support aliasing either (separate in / out pointers)
template <class F, bool TO_AFFINE>
eIcicleError convert_call(const void* input, int size, const VecOpsConfig* cfg, void* output) {
    // point_ops.cu:767-776: null pointers and sizes outside (0, 2^26] are INVALID_ARGUMENT
    if (!input || !output || !cfg) return MBLS_INVALID_ARGUMENT;
    if (size <= 0 || size > POINT_MAX_BATCH) return MBLS_INVALID_ARGUMENT;
    constexpr size_t AFF = PointBytes<F>::AFF, JAC = PointBytes<F>::JAC;
    const size_t in_b = (size_t)size * (TO_AFFINE ? JAC : AFF);
    const size_t out_b = (size_t)size * (TO_AFFINE ? AFF : JAC);
    hipStream_t st = static_cast<hipStream_t>(cfg->stream);
    CtxLease lease(st);
    if (!lease) return lease.error();
    Arena& A = lease->arena;
    const bool in_dev = cfg->is_a_on_device, out_dev = cfg->is_result_on_device;
    eIcicleError er = lease.reserve((in_dev ? 0 : align_up(in_b)) + (out_dev ? 0 : align_up(out_b)));
    if (er != MBLS_SUCCESS) return er;
    const uint8_t* din = static_cast<const uint8_t*>(input);
    uint8_t* dout = static_cast<uint8_t*>(output);
    if (!in_dev) {
        void* t = A.take(in_b);
        MBLS_TRY(hipMemcpyAsync(t, input, in_b, hipMemcpyHostToDevice, st));
        din = static_cast<const uint8_t*>(t);
    }
    if (!out_dev) dout = static_cast<uint8_t*>(A.take(out_b));
    if (TO_AFFINE) {
        const unsigned threads = (unsigned)((size + P2A_RUN - 1) / P2A_RUN);
        hipLaunchKernelGGL(k_jac_to_affine<F>, dim3((threads + 63) / 64), dim3(64), 0, st, din, dout, size);
    } else {
        hipLaunchKernelGGL(k_affine_to_jac<F>, dim3((unsigned)((size + 255) / 256)), dim3(256), 0, st, din, dout, size);
    }
    MBLS_TRY(hipGetLastError());
    if (!out_dev) MBLS_TRY(hipMemcpyAsync(output, dout, out_b, hipMemcpyDeviceToHost, st));
    if (!cfg->is_async || !out_dev) MBLS_TRY(hipStreamSynchronize(st));
    return MBLS_SUCCESS;
}

}  // namespace mbls

using namespace mbls;

extern "C" {

eIcicleError bls12_381_g1_affine_to_projective(const mbls_g1_affine_t* input, int size, const VecOpsConfig* config,
                                               mbls_g1_projective_t* output) {
    return convert_call<Fq, false>(input, size, config, output);
}
eIcicleError bls12_381_g1_projective_to_affine(const mbls_g1_projective_t* input, int size, const VecOpsConfig* config,
                                               mbls_g1_affine_t* output) {
    return convert_call<Fq, true>(input, size, config, output);
}
eIcicleError bls12_381_g2_projective_to_affine(const mbls_g2_projective_t* input, int size, const VecOpsConfig* config,
                                               mbls_g2_affine_t* output) {
    return convert_call<Fq2, true>(input, size, config, output);
}

}  // extern "C"
