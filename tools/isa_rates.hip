// tools/isa_rates.hip -- gfx950 issue rates of the instructions a multiprecision product can be
// built from (32x32 integer mads, FP64 FMAs with exact splits, 64-bit adds, 24-bit and
// dot-product forms, integer / FP64 MFMA), to price the arithmetic engine options in DESIGN.md.
// Each kernel runs 8 independent chains per lane at 4 waves per SIMD; the rate is reported as
// SIMD cycles per wave-instruction at the measured kernel time (clock from --mhz, default 2400).
// Build: hipcc --offload-arch=gfx950 -O3 isa_rates.hip -o isa_rates
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef double v4d __attribute__((ext_vector_type(4)));

enum Op { MAD64, FMA64, MUL64F, ADD64F, LSHLADD64, ADDCO, MULHI, MULLO, MAD24, MULHI24, DOT2U16, ADDU32, CVTF64U32,
          MFMA_I8_16, MFMA_I8_32, MFMA_F64_16, NOPS };
static const char* NAMES[NOPS] = {"v_mad_u64_u32", "v_fma_f64", "v_mul_f64", "v_add_f64", "v_lshl_add_u64",
                                  "v_add_co_u32", "v_mul_hi_u32", "v_mul_lo_u32", "v_mad_u32_u24", "v_mul_hi_u32_u24",
                                  "v_dot2_u32_u16", "v_add_u32", "v_cvt_f64_u32",
                                  "v_mfma_i32_16x16x64_i8", "v_mfma_i32_32x32x32_i8", "v_mfma_f64_16x16x4_f64"};

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint64_t* out, uint32_t seed, int iters) {
    const uint32_t x = seed ^ threadIdx.x, y = x * 2654435761u + 7;
    uint64_t s = 0;
    if constexpr (OP == MAD64) {
        uint64_t a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = x + k;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
                asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a[k]) : "v"(x + k), "v"(y) : "s40", "s41");
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s ^= a[k];
    } else if constexpr (OP == FMA64 || OP == MUL64F || OP == ADD64F) {
        double a[8];
        const double b = (double)x, c = (double)y;
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = (double)(x + k);
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if constexpr (OP == FMA64) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(c));
                if constexpr (OP == MUL64F) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(a[k]) : "v"(b));
                if constexpr (OP == ADD64F) asm volatile("v_add_f64 %0, %1, %0" : "+v"(a[k]) : "v"(b));
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s ^= __double_as_longlong(a[k]);
    } else if constexpr (OP == LSHLADD64) {
        uint64_t a[8];
        const uint64_t b = ((uint64_t)y << 32) | x;
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = x + k;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(a[k]) : "v"(b));
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s ^= a[k];
    } else if constexpr (OP == MFMA_I8_16 || OP == MFMA_I8_32) {
        v4i a = {(int)x, (int)y, (int)(x + 1), (int)(y + 1)}, b = {(int)y, (int)x, 3, 5};
        typedef int v16i __attribute__((ext_vector_type(16)));
        v4i c4[4] = {};
        v16i c16[4] = {};
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if constexpr (OP == MFMA_I8_16) c4[k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c4[k], 0, 0, 0);
                else c16[k] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c16[k], 0, 0, 0);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (OP == MFMA_I8_16) s ^= (uint32_t)(c4[k][0] ^ c4[k][3]);
            else s ^= (uint32_t)(c16[k][0] ^ c16[k][15]);
        }
    } else if constexpr (OP == MFMA_F64_16) {
        v4d c[4] = {};
        const double a = (double)x, b = (double)y;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) s ^= __double_as_longlong(c[k][0] + c[k][3]);
    } else if constexpr (OP == CVTF64U32) {
        double a[8];
        uint32_t u[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = x + k;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a[k]) : "v"(u[k]));
                u[k] = (uint32_t)__double_as_longlong(a[k]);
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s ^= u[k];
    } else {
        uint32_t a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = x + k;
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if constexpr (OP == ADDCO) asm volatile("v_add_co_u32 %0, s[40:41], %1, %0" : "+v"(a[k]) : "v"(y) : "s40", "s41");
                if constexpr (OP == MULHI) asm volatile("v_mul_hi_u32 %0, %1, %0" : "+v"(a[k]) : "v"(y));
                if constexpr (OP == MULLO) asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(a[k]) : "v"(y));
                if constexpr (OP == MAD24) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(a[k]) : "v"(x), "v"(y));
                if constexpr (OP == MULHI24) asm volatile("v_mul_hi_u32_u24 %0, %1, %0" : "+v"(a[k]) : "v"(y));
                if constexpr (OP == DOT2U16) asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(a[k]) : "v"(x), "v"(y));
                if constexpr (OP == ADDU32) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[k]) : "v"(y));
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s ^= a[k];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// shader clock during a busy loop: s_memtime (core clock) against s_memrealtime (100 MHz)
__global__ __launch_bounds__(256) void k_clock(uint64_t* out, int iters) {
    const uint64_t t0 = clock64(), r0 = wall_clock64();
    uint32_t a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = threadIdx.x + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_add_u32 %0, %1, %0" : "+v"(a[k]) : "v"(i));
    }
    const uint64_t t1 = clock64(), r1 = wall_clock64();
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s ^= a[k];
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = s;
    }
}

template <int OP>
static double run(uint64_t* out, int blocks, int iters) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u, iters);  // warm
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 2u, iters);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

template <int OP>
static void report(uint64_t* out, int blocks, int iters, double mhz, int simds) {
    const double ms = run<OP>(out, blocks, iters);
    const int chains = (OP == MFMA_I8_16 || OP == MFMA_I8_32 || OP == MFMA_F64_16) ? 4 : 8;
    const double winst = (double)blocks * 4 * iters * chains;  // wave-instructions
    const double cyc = ms * 1e-3 * mhz * 1e6 * simds / winst;
    printf("%-24s %8.3f ms  %6.2f cycles per wave-instruction per SIMD\n", NAMES[OP], ms, cyc);
}

int main(int argc, char** argv) {
    double mhz = 2400;
    for (int i = 1; i + 1 < argc; ++i)
        if (!strcmp(argv[i], "--mhz")) mhz = atof(argv[i + 1]);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int simds = prop.multiProcessorCount * 4;
    const int blocks = prop.multiProcessorCount * 4;  // 4 waves per SIMD
    uint64_t* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 8));
    printf("%s, %d CUs, clock assumed %.0f MHz\n", prop.gcnArchName, prop.multiProcessorCount, mhz);
    const int it = 65536, itm = 16384;
    for (int w = 0; w < 20; ++w) run<ADDU32>(out, blocks, it);  // clocks up before the first timed op
    {
        hipLaunchKernelGGL(k_clock, dim3(blocks), dim3(256), 0, 0, out, it);
        uint64_t h[3];
        CK(hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost));
        const double m = (double)h[0] / ((double)h[1] / 100.0);
        printf("measured shader clock %.0f MHz (s_memtime %llu ticks over %llu realtime ticks)\n", m,
               (unsigned long long)h[0], (unsigned long long)h[1]);
        if (mhz == 2400 && m > 500 && m < 3000) mhz = m;
    }
    report<MAD64>(out, blocks, it, mhz, simds);
    report<FMA64>(out, blocks, it, mhz, simds);
    report<MUL64F>(out, blocks, it, mhz, simds);
    report<ADD64F>(out, blocks, it, mhz, simds);
    report<LSHLADD64>(out, blocks, it, mhz, simds);
    report<ADDCO>(out, blocks, it, mhz, simds);
    report<MULHI>(out, blocks, it, mhz, simds);
    report<MULLO>(out, blocks, it, mhz, simds);
    report<MAD24>(out, blocks, it, mhz, simds);
    report<MULHI24>(out, blocks, it, mhz, simds);
    report<DOT2U16>(out, blocks, it, mhz, simds);
    report<ADDU32>(out, blocks, it, mhz, simds);
    report<CVTF64U32>(out, blocks, it, mhz, simds);
    report<MFMA_I8_16>(out, blocks, itm, mhz, simds);
    report<MFMA_I8_32>(out, blocks, itm, mhz, simds);
    report<MFMA_F64_16>(out, blocks, itm, mhz, simds);
    report<ADDU32>(out, blocks, it, mhz, simds);
    report<MAD64>(out, blocks, it, mhz, simds);
    CK(hipFree(out));
    return 0;
}
