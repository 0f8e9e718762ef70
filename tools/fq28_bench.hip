// tools/fq28_bench.hip -- radix-2^28 Fq (csrc/mbls_fq28.hpp) against the 32-bit FIPS path:
//   1. bit-exactness of products, squares, lazy product sums, subtraction chains and the
//      conversions, on random canonical Montgomery words (to_words(op(unpack(x))) == fips op);
//   2. bit-exactness of the G1 accumulation chain: 16-point chunks of mixed additions (first point
//      free, second by mmadd, exceptional pairs P + P, P - P and identity points), every Jacobian
//      coordinate compared as canonical words with mbls_curve.hpp's jac_madd / jac_mmadd chain;
//   3. throughput at the accumulation's launch bounds (256 threads, 3 waves per SIMD): dependent
//      product chains, and the k_acc_ceiling structure of tools/valu_ceiling.hip in both forms.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../midnight-bls12-381-cuda_amd/csrc fq28_bench.hip -o fq28_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "mbls_curve.hpp"
#include "mbls_fips.hpp"
#include "mbls_fq28.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

using namespace mbls;
using r28::F28;
using r28::J28;

MBLS_DEV void words_of(const Fq& a, uint32_t (&w)[12]) {
#pragma unroll
    for (int i = 0; i < 12; ++i) w[i] = a.v[i];
}
MBLS_DEV F28 U(const Fq& a) {
    uint32_t w[12];
    words_of(a, w);
    return r28::unpack_shift8(w);
}
MBLS_DEV unsigned neq(const F28& a, const Fq& b) {
    uint32_t w[12];
    r28::to_words(a, w);
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) d |= w[i] ^ b.v[i];
    return d != 0;
}

// ---------------------------------------------------------------- 1. field operations
__global__ __launch_bounds__(256) void k_check_field(const uint32_t* in, unsigned* bad, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const Fq a = load<FqCfg>(in + 48 * t), b = load<FqCfg>(in + 48 * t + 12), c = load<FqCfg>(in + 48 * t + 24),
             d = load<FqCfg>(in + 48 * t + 36);
    const F28 ua = U(a), ub = U(b), uc = U(c), ud = U(d);
    unsigned e[8] = {};
    e[0] = neq(ua, a);                                                   // conversion round trip
    e[1] = neq(r28::mul(ua, ub), a * b);                                 // product
    e[2] = neq(r28::sqr(ua), sqr(a));                                    // square
    e[3] = neq(r28::mul2(ua, ub, uc, ud), fips::mul2(a, b, c, d));       // lazy product sum
    // products of in-range operands (< 2p, normalised) as the formulas have them: one unpacked
    // operand (< 256 p) meets a reduced one; two unpacked operands would give < 27 p
    const F28 one = F28::one(), sa = r28::mul(ua, one), sb = r28::mul(ub, one), sc = r28::mul(uc, one);
    const F28 pe = r28::mul(sa, sb), pf = r28::sqr(sc);
    e[4] = neq(r28::sub<r28::B16>(pe, pf), a * b - sqr(c));              // biased subtraction
    e[5] = neq(r28::fold(r28::sub<r28::B32>(pe, r28::x2(pf))), a * b - dbl(sqr(c)));
    e[6] = neq(r28::mul(r28::x4(pe), r28::carry(r28::x2(r28::sub<r28::B16>(pf, pe)))),
               dbl(dbl(a * b)) * dbl(sqr(c) - a * b));                   // unreduced operands
    e[7] = r28::is_zero_mod(r28::sub<r28::B16>(pe, pe)) ? 0u : 1u;        // 0 mod p detection
    for (int k = 0; k < 8; ++k)
        if (e[k]) atomicAdd(&bad[k], 1u);
}

// ---------------------------------------------------------------- 2. accumulation chains
// points: 16 per thread, (x, y) canonical words; the host plants duplicates, negations and
// identities.  Both chains follow k_accumulate's step logic.
__global__ __launch_bounds__(256) void k_check_chain(const uint32_t* pts, unsigned* bad, int n) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    Jacobian<Fq> ref = Jacobian<Fq>::inf();
    J28 acc = J28::inf();
    for (int e = 0; e < 16; ++e) {
        const uint32_t* p = pts + 24 * (16 * t + e);
        const Affine<Fq> q = {load<FqCfg>(p), load<FqCfg>(p + 12)};
        // reference (msm_core.hpp k_accumulate step)
        bool done = false;
        if (e == 1 && !ref.is_inf() && !q.is_inf()) done = jac_mmadd(ref, q, ref);
        if (!done) ref = jac_madd(ref, q);
        // radix 2^28
        if (!q.is_inf()) {
            const F28 qx = U(q.x), qy = U(q.y);
            bool d28 = false;
            if (e == 1 && !acc.is_inf()) d28 = r28::mmadd(acc, qx, qy);
            if (!d28) r28::madd(acc, qx, qy);
        }
    }
    unsigned m = 0;
    if (ref.is_inf() != acc.is_inf()) m |= 1;
    if (!ref.is_inf()) m |= neq(acc.x, ref.x) << 1 | neq(acc.y, ref.y) << 2 | neq(acc.z, ref.z) << 3;
    if (m) atomicAdd(&bad[0], 1u);
    if (ref.is_inf()) atomicAdd(&bad[1], 1u);
    bad[2 + t % 4] = bad[2 + t % 4] | m;
}

// ---------------------------------------------------------------- 3. throughput
template <int MODE>  // 0: FIPS product chain, 1: radix-2^28 product chain
__global__ __launch_bounds__(256, 3) void k_prod_rate(const uint32_t* in, uint32_t* out, int iters) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const Fq a = load<FqCfg>(in + 12 * (t & 1023)), b = load<FqCfg>(in + 12 * ((t * 7 + 3) & 1023));
    if constexpr (MODE == 0) {
        Fq x = a;
        for (int i = 0; i < iters; ++i) x = x * b;
        store<FqCfg>(out + 12 * t, x);
    } else {
        F28 x = U(a);
        const F28 y = U(b);
        for (int i = 0; i < iters; ++i) x = r28::mul(x, y);
        uint32_t w[12];
        r28::to_words(x, w);
#pragma unroll
        for (int k = 0; k < 12; ++k) out[12 * t + k] = w[k];
    }
}

static constexpr int PTS = 64;
template <int MODE>  // k_acc_ceiling of tools/valu_ceiling.hip: 0 FIPS, 1 radix 2^28
__global__ __launch_bounds__(256, 3) void k_acc(const uint8_t* __restrict__ table, uint8_t* __restrict__ partials,
                                                uint32_t chunks_per_thread, uint32_t seed) {
    __shared__ uint4 pts[PTS * 6];
    for (int k = threadIdx.x; k < PTS * 6; k += blockDim.x) pts[k] = reinterpret_cast<const uint4*>(table)[k];
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = seed ^ (tid * 0x9e3779b9u);
    for (uint32_t ch = 0; ch < chunks_per_thread; ++ch) {
        Jacobian<Fq> acc = Jacobian<Fq>::inf();
        J28 a28 = J28::inf();
        for (int e = 0; e < 16; ++e) {
            h = h * 1664525u + 1013904223u;
            const uint32_t idx = (h >> 8) & (PTS - 1);
            Affine<Fq> p;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = pts[idx * 6 + k], ya = pts[idx * 6 + 3 + k];
                p.x.v[4 * k] = xa.x, p.x.v[4 * k + 1] = xa.y, p.x.v[4 * k + 2] = xa.z, p.x.v[4 * k + 3] = xa.w;
                p.y.v[4 * k] = ya.x, p.y.v[4 * k + 1] = ya.y, p.y.v[4 * k + 2] = ya.z, p.y.v[4 * k + 3] = ya.w;
            }
            const Affine<Fq> q = (h & 1) ? aff_neg(p) : p;
            if constexpr (MODE == 0) {
                bool done = false;
                if (e == 1 && !acc.is_inf() && !q.is_inf()) done = jac_mmadd(acc, q, acc);
                if (!done) acc = jac_madd(acc, q);
            } else {
                if (!q.is_inf()) {
                    const F28 qx = U(q.x), qy = U(q.y);
                    bool d = false;
                    if (e == 1 && !a28.is_inf()) d = r28::mmadd(a28, qx, qy);
                    if (!d) r28::madd(a28, qx, qy);
                }
            }
        }
        if constexpr (MODE == 1) {
            uint32_t w[12];
            r28::to_words(a28.x, w);
#pragma unroll
            for (int k = 0; k < 12; ++k) acc.x.v[k] = w[k];
            r28::to_words(a28.y, w);
#pragma unroll
            for (int k = 0; k < 12; ++k) acc.y.v[k] = w[k];
            r28::to_words(a28.z, w);
#pragma unroll
            for (int k = 0; k < 12; ++k) acc.z.v[k] = w[k];
        }
        store_jac<Fq>(partials, (size_t)tid * chunks_per_thread + ch, acc);
    }
}

// ---------------------------------------------------------------- host
static uint32_t rs = 0x12345678u;
static uint32_t rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 17;
    rs ^= rs << 5;
    return rs;
}
static const uint32_t PW[12] = {0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
static void rand_fq(uint32_t* w) {  // uniform-ish canonical (< p): top word below p's
    for (int i = 0; i < 12; ++i) w[i] = rnd();
    w[11] %= PW[11];
}
static void neg_fq(uint32_t* w) {  // p - w (w != 0)
    uint64_t br = 0;
    for (int i = 0; i < 12; ++i) {
        uint64_t d = (uint64_t)PW[i] - w[i] - br;
        w[i] = (uint32_t)d;
        br = (d >> 63) & 1;
    }
}

template <class L>
static float time_ms(L launch, int reps = 5) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> v(reps);
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&v[r], a, b));
    }
    std::sort(v.begin(), v.end());
    return v[reps / 2];
}

int main() {
    unsigned* d_bad;
    CK(hipMalloc(&d_bad, 64 * sizeof(unsigned)));
    // 1. field ops
    const int nf = 1 << 18;
    std::vector<uint32_t> f(48 * (size_t)nf);
    for (int i = 0; i < 4 * nf; ++i) rand_fq(&f[12 * (size_t)i]);
    for (int k = 0; k < 12; ++k) f[k] = 0;                       // a = 0
    for (int k = 0; k < 12; ++k) f[48 + k] = PW[k] - (k == 0);   // a = p - 1
    uint32_t* d_f;
    CK(hipMalloc(&d_f, f.size() * 4));
    CK(hipMemcpy(d_f, f.data(), f.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_bad, 0, 64 * sizeof(unsigned)));
    hipLaunchKernelGGL(k_check_field, dim3(nf / 256), dim3(256), 0, 0, d_f, d_bad, nf);
    unsigned bad[64];
    CK(hipMemcpy(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost));
    printf("{\"field_cases\": %d, \"field_mismatch\": [%u, %u, %u, %u, %u, %u, %u, %u]", nf, bad[0], bad[1], bad[2],
           bad[3], bad[4], bad[5], bad[6], bad[7]);
    // 2. chains with planted exceptional cases
    const int nc = 1 << 16;
    std::vector<uint32_t> pts(24 * 16 * (size_t)nc);
    for (size_t i = 0; i < 16 * (size_t)nc; ++i) {
        rand_fq(&pts[24 * i]);
        rand_fq(&pts[24 * i + 12]);
    }
    int planted = 0;
    for (int t = 0; t < nc; ++t) {
        uint32_t* c = &pts[24 * 16 * (size_t)t];
        const int kind = t % 8;
        if (kind == 1) {  // second point equal to the first: mmadd refuses, madd doubles
            std::copy(c, c + 24, c + 24);
        } else if (kind == 2) {  // second point the negation of the first: infinity, then restart
            std::copy(c, c + 24, c + 24);
            neg_fq(c + 24 + 12);
        } else if (kind == 3) {  // a later point equal to an earlier one cannot be planted (acc is Jacobian)
            std::fill(c + 24 * 5, c + 24 * 6, 0u);  // identity point in the middle
            std::fill(c, c + 24, 0u);               // and first
        } else if (kind == 4) {
            std::fill(c + 24, c + 48, 0u);  // identity as the second point
        } else {
            continue;
        }
        ++planted;
    }
    uint32_t* d_p;
    CK(hipMalloc(&d_p, pts.size() * 4));
    CK(hipMemcpy(d_p, pts.data(), pts.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemset(d_bad, 0, 64 * sizeof(unsigned)));
    hipLaunchKernelGGL(k_check_chain, dim3(nc / 256), dim3(256), 0, 0, d_p, d_bad, nc);
    CK(hipMemcpy(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost));
    printf(",\n \"chain_cases\": %d, \"chain_planted\": %d, \"chain_mismatch\": %u, \"chain_infinity\": %u, "
           "\"chain_mismatch_bits\": [%u, %u, %u, %u]",
           nc, planted, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5]);
    // 3. throughput
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int blocks = prop.multiProcessorCount * 3 * 4;
    uint32_t* d_o;
    CK(hipMalloc(&d_o, (size_t)blocks * 256 * 12 * 4 * 64));
    const int it = 2048;
    const float t0 = time_ms([&] { hipLaunchKernelGGL(k_prod_rate<0>, dim3(blocks), dim3(256), 0, 0, d_f, d_o, it); });
    const float t1 = time_ms([&] { hipLaunchKernelGGL(k_prod_rate<1>, dim3(blocks), dim3(256), 0, 0, d_f, d_o, it); });
    const double prods = (double)blocks * 256 * it;
    printf(",\n \"fips_G_products_per_s\": %.2f, \"r28_G_products_per_s\": %.2f", prods / (t0 * 1e-3) / 1e9,
           prods / (t1 * 1e-3) / 1e9);
    const uint32_t threads = prop.multiProcessorCount * 3 * 256 * 4, per = 4;
    uint8_t* d_part;
    CK(hipMalloc(&d_part, (size_t)threads * per * 144));
    const float a0 = time_ms([&] {
        hipLaunchKernelGGL(k_acc<0>, dim3(threads / 256), dim3(256), 0, 0, (const uint8_t*)d_f, d_part, per, 9u);
    });
    const float a1 = time_ms([&] {
        hipLaunchKernelGGL(k_acc<1>, dim3(threads / 256), dim3(256), 0, 0, (const uint8_t*)d_f, d_part, per, 9u);
    });
    const double contrib = (double)threads * per * 16;
    printf(",\n \"acc_fips_ms_per_2^24_contrib\": %.4f, \"acc_r28_ms_per_2^24_contrib\": %.4f, \"acc_speedup\": %.4f}\n",
           a0 / contrib * 16777216.0, a1 / contrib * 16777216.0, a0 / a1);
    return 0;
}
