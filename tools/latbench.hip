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
__global__ void k_rf(uint32_t* out, const uint32_t* in, int n) {
    RFq x = rf_in(in, 0), y = rf_in(in, 1);
    for (int i = 0; i < n; ++i) {
        if constexpr (OP == 0) x = x * y;
        if constexpr (OP == 1) x = x + y;
        if constexpr (OP == 2) x = x - y;
    }
    out[threadIdx.x] = x.v;
}

template <int OP>
__global__ void k_wave(uint32_t* out, const uint32_t* in, int n) {
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
__global__ void k_lane(uint32_t* out, const uint32_t* in, int n) {
    Fq x = load<FqCfg>(in), y = load<FqCfg>(in + 12);
    for (int i = 0; i < n; ++i) {
        if constexpr (OP == 0) x = fips::mul(x, y);
        if constexpr (OP == 1) x = x + y;
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
    run("wave jdbl", k_wave<0>, out, in, 2000);
    run("wave jadd", k_wave<1>, out, in, 2000);
    run("row jac_dbl", k_wave<2>, out, in, 2000);
    run("row jac_add", k_wave<3>, out, in, 2000);
    return 0;
}
