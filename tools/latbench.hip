// tools/latbench.hip -- latency of the serial-chain primitives on ONE wave (the MSM tail's unit
// of work): a chain of N dependent operations, time / N.  Values are arbitrary field words
// (timing only).  Build: hipcc --offload-arch=gfx950 -O3 -I../midnight-bls12-381-cuda_amd/csrc latbench.hip -o latbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "mbls_curve.hpp"
#include "mbls_fips.hpp"
#include "mbls_rowfield.hpp"
#include "mbls_wavepoint.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using namespace mbls;

MBLS_DEV RFq rf_in(const uint32_t* in, int k) {
    const uint32_t j = rowdpp::lane16();
    return {j < 12 ? in[12 * k + j] : 0u};
}

template <int OP>
__global__ __launch_bounds__(64) void k_rf(uint32_t* out, const uint32_t* in, int n) {
    RFq x = rf_in(in, 0), y = rf_in(in, 1);
    for (int i = 0; i < n; ++i) {
        if constexpr (OP == 0) x = x * y;
        if constexpr (OP == 1) x = x + y;
        if constexpr (OP == 2) x = x - y;
    }
    out[threadIdx.x] = x.v;
}

template <int OP>
__global__ __launch_bounds__(64) void k_wave(uint32_t* out, const uint32_t* in, int n) {
    Jacobian<RFq> p{rf_in(in, 0), rf_in(in, 1), rf_in(in, 2)}, q{rf_in(in, 3), rf_in(in, 4), rf_in(in, 5)};
    for (int i = 0; i < n; ++i) {
        if constexpr (OP == 0) p = wave::jdbl(p);
        if constexpr (OP == 1) p = wave::jadd(p, q);
        if constexpr (OP == 2) p = jac_dbl(p);  // row mode: one point per row
        if constexpr (OP == 3) p = jac_add(p, q);
    }
    out[threadIdx.x] = p.x.v ^ p.y.v ^ p.z.v;
}

template <int OP>
__global__ __launch_bounds__(64) void k_lane(uint32_t* out, const uint32_t* in, int n) {
    Fq x = load<FqCfg>(in), y = load<FqCfg>(in + 12);
    for (int i = 0; i < n; ++i) {
        if constexpr (OP == 0) x = fips::mul(x, y);
        if constexpr (OP == 1) x = x + y;
        if constexpr (OP == 2) x = inv(x) + y;  // binary GCD inversion chain
        if constexpr (OP == 4) {                // the same on wave-uniform (SGPR, scalar-ALU) operands
#pragma unroll
            for (int k = 0; k < 12; ++k) x.v[k] = __builtin_amdgcn_readfirstlane(x.v[k]);
            Fq z;
            binv::inverse<12>(z.v, x.v, FqCfg::MOD, FqCfg::NINV);
            x = z + y;
        }
        if constexpr (OP == 3) {                // the (x, y, 1) normalisation of one point
            Jacobian<Fq> p{x, y, x + y};
            Affine<Fq> a = jac_to_affine(p);
            x = from_mont(a.x) + from_mont(a.y);
        }
    }
    store<FqCfg>(out + 12 * threadIdx.x, x);
}

// row ops vs lane-mode Fq on random canonical inputs: 64 lanes = 4 rows, each row one element
__global__ void k_check(unsigned* bad, const uint32_t* in, int iters) {
    const uint32_t j = rowdpp::lane16(), row = (threadIdx.x >> 4) + 4 * blockIdx.x;
    RFq a = {j < 12 ? in[12 * (2 * row) + j] : 0u}, b = {j < 12 ? in[12 * (2 * row + 1) + j] : 0u};
    Fq la = load<FqCfg>(in + 12 * (2 * row)), lb = load<FqCfg>(in + 12 * (2 * row + 1));
    for (int it = 0; it < iters; ++it) {
        RFq r[5] = {a + b, a - b, b - a, a * b, a + a};
        Fq l[5] = {la + lb, la - lb, lb - la, la * lb, la + la};
        for (int k = 0; k < 5; ++k) {
            const uint32_t want = j < 12 ? l[k].v[j] : 0u;
            if (r[k].v != want) atomicAdd(bad + k, 1u);
        }
        a = r[3] + r[1];
        b = r[2] - r[4];
        la = l[3] + l[1];
        lb = l[2] - l[4];
        if (it % 7 == 3) { b = a; lb = la; }  // equal operands: a - b = 0, b - a = 0
    }
}

// pieces of one binary-GCD outer step, chained: OP 0 the 30 inner steps, 1 lincomb_shift,
// 2 lincomb_mod, 3 bitlen + top33 approximations
template <int OP>
__global__ __launch_bounds__(64) void k_binv_part(uint32_t* out, const uint32_t* in, int n) {
    uint32_t a[12], b[12];
    for (int i = 0; i < 12; ++i) {
        a[i] = in[i];
        b[i] = in[12 + i];
    }
    uint64_t xa = ((uint64_t)a[1] << 32) | a[0], xb = ((uint64_t)b[1] << 32) | b[0];
    int64_t f = 12345, g = -54321;
    for (int it = 0; it < n; ++it) {
        if constexpr (OP == 0) {
            uint64_t F0 = 1, F1 = 1ull << 32;
#pragma unroll
            for (int j = 0; j < binv::K; ++j) {
                const bool odd = (xa & 1) != 0;
                const bool lt = xa < xb;
                const bool sw = odd && lt;
                const uint64_t d = lt ? xb - xa : xa - xb;
                const uint64_t G0 = sw ? F1 : F0, G1 = sw ? F0 : F1;
                xb = sw ? xa : xb;
                xa = (odd ? d : xa) >> 1;
                F0 = odd ? G0 - G1 : G0;
                F1 = G1 << 1;
            }
            xa ^= F0 + F1 + 3;
        } else if constexpr (OP == 1) {
            uint32_t r[12];
            if (binv::lincomb_shift<12>(r, a, b, f, g)) f = -f;
            for (int i = 0; i < 12; ++i) a[i] = r[i] ^ in[i];
        } else if constexpr (OP == 2) {
            uint32_t r[12];
            binv::lincomb_mod<12>(r, a, b, f, g, FqCfg::MOD, FqCfg::NINV);
            for (int i = 0; i < 12; ++i) a[i] = r[i];
        } else {
            const int nl = binv::bitlen_or<12>(a, b);
            const int nn = nl > 64 ? nl : 64;
            xa += (a[0] & 0x7fffffffu) | (binv::top33<12>(a, nn - 33) << 31);
            xb += (b[0] & 0x7fffffffu) | (binv::top33<12>(b, nn - 33) << 31);
            a[(it & 3)] ^= (uint32_t)xa;
        }
    }
    uint32_t o = (uint32_t)xa ^ (uint32_t)xb;
    for (int i = 0; i < 12; ++i) o ^= a[i];
    out[threadIdx.x] = o;
}

template <class K>
static void run(const char* name, K kern, uint32_t* out, const uint32_t* in, int n) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kern, 1, 64, 0, 0, out, in, 4);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, 1, 64, 0, 0, out, in, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.3f us/op  (%d ops, %.3f ms)\n", name, ms * 1e3 / n, n, ms);
}

int main() {
    uint32_t *in, *out;
    CK(hipMalloc(&in, 4 * 12 * 8));
    CK(hipMalloc(&out, 4 * 12 * 64));
    uint32_t h[96];
    srand(7);
    for (int i = 0; i < 96; ++i) h[i] = (uint32_t)rand() * 2654435761u;
    for (int k = 0; k < 8; ++k) h[12 * k + 11] &= 0x0fffffff;
    CK(hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice));
    {
        const int rows = 4096;
        uint32_t* rin;
        CK(hipMalloc(&rin, 4 * 12 * 2 * rows));
        uint32_t* hr = (uint32_t*)malloc(4 * 12 * 2 * rows);
        for (int i = 0; i < 12 * 2 * rows; ++i) hr[i] = (uint32_t)rand() * 2654435761u ^ (uint32_t)rand();
        for (int e = 0; e < 2 * rows; ++e) {
            hr[12 * e + 11] %= 0x1a0111eau;  // < p
            if (e % 97 == 0) for (int k = 0; k < 12; ++k) hr[12 * e + k] = 0;  // zero operands
        }
        CK(hipMemcpy(rin, hr, 4 * 12 * 2 * rows, hipMemcpyHostToDevice));
        unsigned* bad;
        CK(hipMalloc(&bad, 32));
        CK(hipMemset(bad, 0, 32));
        hipLaunchKernelGGL(k_check, rows / 4, 64, 0, 0, bad, rin, 64);
        unsigned hb[5];
        CK(hipMemcpy(hb, bad, 20, hipMemcpyDeviceToHost));
        printf("row vs lane mismatches (add, sub, rsub, mul, dbl) over %d x 64: %u %u %u %u %u\n", rows, hb[0], hb[1],
               hb[2], hb[3], hb[4]);
        free(hr);
    }
    run("row Fq mul", k_rf<0>, out, in, 20000);
    run("row Fq add", k_rf<1>, out, in, 20000);
    run("row Fq sub", k_rf<2>, out, in, 20000);
    run("lane Fq mul (fips)", k_lane<0>, out, in, 20000);
    run("lane Fq add", k_lane<1>, out, in, 20000);
    run("lane Fq inverse (binary GCD)", k_lane<2>, out, in, 200);
    run("lane jac_to_affine + from_mont", k_lane<3>, out, in, 200);
    run("lane Fq inverse, uniform operands", k_lane<4>, out, in, 200);
    run("binv: 30 inner steps", k_binv_part<0>, out, in, 2000);
    run("binv: lincomb_shift", k_binv_part<1>, out, in, 2000);
    run("binv: lincomb_mod", k_binv_part<2>, out, in, 2000);
    run("binv: bitlen + top33 x2", k_binv_part<3>, out, in, 2000);
    run("wave jdbl", k_wave<0>, out, in, 2000);
    run("wave jadd", k_wave<1>, out, in, 2000);
    run("row jac_dbl", k_wave<2>, out, in, 2000);
    run("row jac_add", k_wave<3>, out, in, 2000);
    return 0;
}
