// tools/microbench.hip -- gfx950 roof probes used for the design decisions in DESIGN.md:
//   * v_mad_u64_u32 issue rate (the multiprecision multiply primitive),
//   * Fr / Fq Montgomery-multiply rate of mbls_field.hpp,
//   * streaming copy bandwidth (achievable HBM roof).
// Build: hipcc --offload-arch=gfx950 -O3 -I../midnight-bls12-381-cuda_amd/csrc microbench.hip -o microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "mbls_field.hpp"
#include "mbls_fips.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

using namespace mbls;

__global__ void k_mad(uint64_t* out, uint32_t seed, int iters) {
    uint32_t x = seed ^ threadIdx.x;
    uint64_t acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = x + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = (uint64_t)(uint32_t)acc[k] * (x + k) + (acc[k] >> 32);
    }
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s ^= acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// OP 0: CIOS operator*, 1: fips::mul, 2: fips::sqr
template <class C, int OP>
MBLS_DEV Fp<C> opf(const Fp<C>& a, const Fp<C>& b) {
    if constexpr (OP == 0) return a * b;
    if constexpr (OP == 1) return fips::mul(a, b);
    return fips::sqr(a);
}

// correctness: compare fips mul/sqr with CIOS on a*b and a*a; count mismatches
template <class C>
__global__ void k_check(unsigned* bad, const uint32_t* in) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fp<C> a = load<C>(in + C::N * (tid & 1023));
    Fp<C> b = load<C>(in + C::N * ((tid * 7 + 3) & 1023));
    for (int it = 0; it < 8; ++it) {
        Fp<C> r0 = a * b, r1 = fips::mul(a, b), s0 = a * a, s1 = fips::sqr(a);
        if (!(r0 == r1)) atomicAdd(bad, 1u);
        if (!(s0 == s1)) atomicAdd(bad + 1, 1u);
        a = r0;
        b = s0 + b;
    }
}

template <class C, int CH, int OP = 0>
__global__ void k_mont(uint32_t* out, const uint32_t* in, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fp<C> x[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
        x[k] = load<C>(in + C::N * ((tid + k) & 1023));
    }
    Fp<C> y = load<C>(in + C::N * 1024);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < CH; ++k) x[k] = opf<C, OP>(x[k], y);
    }
    Fp<C> s = x[0];
#pragma unroll
    for (int k = 1; k < CH; ++k) s = s + x[k];
    store<C>(out + C::N * tid, s);
}

// inversion throughput: OP 0 binary GCD inv(), OP 1 Fermat
template <class C, int OP>
__global__ void k_inv(uint32_t* out, const uint32_t* in, int iters) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fp<C> x = load<C>(in + C::N * (tid & 1023));
    for (int i = 0; i < iters; ++i) {
        if constexpr (OP == 0) x = inv(x); else x = inv_fermat(x);
        x.v[0] ^= 1;
    }
    store<C>(out + C::N * tid, x);
}

__global__ void k_copy(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += stride) dst[i] = src[i];
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    printf("device %s CUs %d clock %d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;

    // ---- mad rate
    {
        int blocks = 256 * 8, threads = 256, iters = 4096;
        uint64_t* out;
        CK(hipMalloc(&out, sizeof(uint64_t) * blocks * threads));
        hipLaunchKernelGGL(k_mad, blocks, threads, 0, 0, out, 1u, 16);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_mad, blocks, threads, 0, 0, out, 1u, iters);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        double mads = (double)blocks * threads * iters * 8;
        printf("mad_u64_u32: %.3f ms, %.3f Tmad/s (%.1f mad/clk/CU @2.4GHz)\n", ms, mads / ms / 1e9,
               mads / (ms * 1e-3) / 256 / 2.4e9);
        CK(hipFree(out));
    }
    // ---- Montgomery mul rate
    {
        uint32_t* in;
        uint32_t* out;
        int blocks = 256 * 8, threads = 256, iters = 256;
        CK(hipMalloc(&in, 4 * 12 * 2048));
        CK(hipMalloc(&out, 4 * 12 * (size_t)blocks * threads));
        uint32_t* h = (uint32_t*)malloc(4 * 12 * 2048);
        for (int i = 0; i < 12 * 2048; ++i) h[i] = (uint32_t)rand();
        for (int i = 0; i < 2048; ++i) { h[12 * i + 11] &= 0x0fffffff; }
        // keep Fr-view values < r too: top word of each 8-word group small
        for (int i = 0; i < 12 * 2048 / 8; ++i) h[8 * i + 7] &= 0x0fffffff;
        CK(hipMemcpy(in, h, 4 * 12 * 2048, hipMemcpyHostToDevice));
#define RUN_MONT(C, CH, OP)                                                                          \
        {                                                                                            \
            hipLaunchKernelGGL((k_mont<C, CH, OP>), blocks, threads, 0, 0, out, in, 4);              \
            CK(hipDeviceSynchronize());                                                              \
            CK(hipEventRecord(e0));                                                                  \
            hipLaunchKernelGGL((k_mont<C, CH, OP>), blocks, threads, 0, 0, out, in, iters);          \
            CK(hipEventRecord(e1));                                                                  \
            CK(hipEventSynchronize(e1));                                                             \
            CK(hipEventElapsedTime(&ms, e0, e1));                                                    \
            double muls = (double)blocks * threads * iters * CH;                                     \
            printf(#C " op%d x%d chains: %.3f ms, %.2f Gmul/s\n", OP, CH, ms, muls / ms / 1e6);      \
        }
        {
            unsigned* bad;
            CK(hipMalloc(&bad, 16));
            CK(hipMemset(bad, 0, 16));
            hipLaunchKernelGGL(k_check<FrCfg>, 256, 256, 0, 0, bad, in);
            hipLaunchKernelGGL(k_check<FqCfg>, 256, 256, 0, 0, bad + 2, in);
            unsigned hb[4];
            CK(hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost));
            printf("fips check mismatches: Fr mul %u sqr %u | Fq mul %u sqr %u (of %d each)\n", hb[0], hb[1], hb[2],
                   hb[3], 256 * 256 * 8);
        }
        // occupancy sweep (dynamic LDS caps the resident 256-thread blocks per CU at 1, 2, 3, 4):
        // Fq fips::mul throughput with 1 and 2 independent chains per thread -> latency exposure
        for (int occ = 1; occ <= 4; ++occ) {
            size_t lds = (160 * 1024) / occ - 1024;
            for (int ch = 1; ch <= 2; ++ch) {
                auto kern = ch == 1 ? k_mont<FqCfg, 1, 1> : k_mont<FqCfg, 2, 1>;
                hipLaunchKernelGGL(kern, blocks, threads, lds, 0, out, in, 4);
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(kern, blocks, threads, lds, 0, out, in, iters);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms, e0, e1));
                double muls = (double)blocks * threads * iters * ch;
                printf("occ %d waves/SIMD Fq fips mul x%d chains: %.3f ms, %.2f Gmul/s\n", occ, ch, ms, muls / ms / 1e6);
            }
        }
        for (int op = 0; op < 2; ++op) {
            auto kern = op == 0 ? k_inv<FqCfg, 0> : k_inv<FqCfg, 1>;
            int it = 8;
            hipLaunchKernelGGL(kern, blocks, threads, 0, 0, out, in, 1);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, blocks, threads, 0, 0, out, in, it);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            double n = (double)blocks * threads * it;
            printf("Fq inverse (%s): %.3f ms, %.3f Ginv/s\n", op == 0 ? "binary GCD" : "Fermat", ms, n / ms / 1e6);
        }
        RUN_MONT(FrCfg, 1, 0)
        RUN_MONT(FrCfg, 2, 0)
        RUN_MONT(FrCfg, 1, 1)
        RUN_MONT(FrCfg, 2, 1)
        RUN_MONT(FrCfg, 1, 2)
        RUN_MONT(FrCfg, 2, 2)
        RUN_MONT(FqCfg, 1, 0)
        RUN_MONT(FqCfg, 2, 0)
        RUN_MONT(FqCfg, 1, 1)
        RUN_MONT(FqCfg, 2, 1)
        RUN_MONT(FqCfg, 1, 2)
        RUN_MONT(FqCfg, 2, 2)
        CK(hipFree(in));
        CK(hipFree(out));
        free(h);
    }
    // ---- copy bandwidth
    {
        size_t bytes = (size_t)1 << 30;
        uint4 *a, *b;
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&b, bytes));
        CK(hipMemset(a, 1, bytes));
        size_t n = bytes / 16;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_copy, 256 * 16, 256, 0, 0, b, a, n);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
        }
        printf("copy 1 GiB: %.3f ms, %.2f TB/s (read+write)\n", ms, 2.0 * bytes / ms / 1e9);
        CK(hipFree(a));
        CK(hipFree(b));
    }
    return 0;
}
