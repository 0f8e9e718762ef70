// tools/valu_ceiling.hip -- MEASURED VALU ceilings for the two dominant kernels.
//
// The bench line's VALU fractions used to price k_accumulate against a cycle MODEL (8 cycles per
// INT64 wave-instruction, 2 otherwise, 2.4 GHz), which the kernel beat (counter_issue_frac 1.05).
// This program measures instead:
//   * the shader clock during a saturated kernel: clock64() (s_memtime, shader cycles) against
//     wall_clock64() (constant-rate counter, hipDeviceAttributeWallClockRate), per wave;
//   * cycles per wave-instruction for v_mad_u64_u32 alone, v_addc_co_u32 alone and the FIPS
//     pair (mad with carry-out to an SGPR pair + addc of that carry), at 3 waves per SIMD;
//   * k_acc_ceiling: k_accumulate<G1>'s per-contribution arithmetic (madd-2007-bl with the lazy
//     Y3, the chunk's first point free and its second by mmadd-2007-bl, one Jacobian partial
//     stored per 16-point chunk, the point's sign applied) with the SAME code (mbls_curve.hpp),
//     the SAME launch bounds (256 threads, 3 waves per SIMD -> 168 VGPRs) and the points read
//     from LDS as k_accumulate reads its LDS-DMA stage -- but no random HBM gathers, no sorted
//     index stream and no bucket boundaries.  Its time per contribution is the ceiling the
//     accumulation could reach with a perfect memory system;
//   * k_acc28p_ceiling: k_accumulate_r28p<G2>'s arithmetic (round 6: pair-sliced radix-2^28 Fq2,
//     mbls_fq2_28.hpp) -- the same madd / mmadd over lane pairs, 16-point chunks, the same launch
//     bounds, points from LDS;
//   * k_ntt_ceiling: k_ntt_pass's round-5 radix-4 (2 x 2) DIT butterfly body (4 lazy FIPS Fr
//     products, 8 add_2r / sub_2r) register-resident with twiddles from LDS, at the pass's launch
//     bounds; k_ntt29_ceiling: the same body with the round-6 products (mbls_fr29.hpp: radix-2^29
//     limbs, twiddles as w R' limb planes) -- the shipped k_ntt_pass's arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../midnight-bls12-381-cuda_amd/csrc valu_ceiling.hip -o valu_ceiling
// Run:   ./valu_ceiling [contributions_log2 = 24]  (prints one JSON object)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <vector>
#include "mbls_curve.hpp"
#include "mbls_fips.hpp"
#include "mbls_fq28.hpp"
#include "mbls_fr29.hpp"
#include "mbls_fq2_28.hpp"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

using namespace mbls;

// per-wave clock record: [shader clock start, end, wall start, end]
struct Clk {
    unsigned long long c0, c1, w0, w1;
};
MBLS_DEV void clk_begin(unsigned long long& c, unsigned long long& w) {
    w = wall_clock64();
    c = clock64();
}
MBLS_DEV void clk_end(Clk* rec, unsigned long long c0, unsigned long long w0) {
    const unsigned long long c1 = clock64(), w1 = wall_clock64();
    if ((threadIdx.x & 63) == 0) rec[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = Clk{c0, c1, w0, w1};
}

// ---------------------------------------------------------------------------------- ISA rates
// OP 0: v_mad_u64_u32 only; 1: v_addc_co_u32 only; 2: FIPS pair (mad -> SGPR carry -> addc)
template <int OP>
__global__ __launch_bounds__(256, 3) void k_isa(uint64_t* out, Clk* rec, uint32_t seed, int iters) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    const uint32_t x = seed ^ threadIdx.x, y = x * 2654435761u + 7;
    uint64_t a[8];
    uint32_t cnt[8], hi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = x + k;
        cnt[k] = y ^ k;
        hi[k] = x * k;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint64_t c;
            if constexpr (OP == 0)
                asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(a[k]), "=&s"(c) : "v"(x + k), "v"(y));
            if constexpr (OP == 1)
                asm volatile("v_add_co_u32 %0, %1, %0, %2\n\tv_addc_co_u32 %3, %1, 0, %3, %1"
                             : "+v"(cnt[k]), "=&s"(c), "+v"(hi[k]) : "v"(x + k));
            if constexpr (OP == 2)
                asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32 %2, %1, 0, %2, %1"
                             : "+v"(a[k]), "=&s"(c), "+v"(cnt[k]) : "v"(x + k), "v"(y));
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s ^= a[k] ^ cnt[k] ^ hi[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    clk_end(rec, c0, w0);
}

// ------------------------------------------------------------------ k_accumulate<G1> ceiling
static constexpr int PTS = 64;  // LDS point table (96 B each)

template <int CHUNK>
__global__ __launch_bounds__(256, 3) void k_acc_ceiling(const uint8_t* __restrict__ table, uint8_t* __restrict__ partials,
                                                        Clk* rec, uint32_t chunks_per_thread, uint32_t seed) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 pts[PTS * 6];
    for (int k = threadIdx.x; k < PTS * 6; k += blockDim.x) pts[k] = reinterpret_cast<const uint4*>(table)[k];
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = seed ^ (tid * 0x9e3779b9u);
    for (uint32_t ch = 0; ch < chunks_per_thread; ++ch) {
        Jacobian<Fq> acc = Jacobian<Fq>::inf();
        for (int e = 0; e < CHUNK; ++e) {
            h = h * 1664525u + 1013904223u;  // the point index / sign stream (LCG)
            const uint32_t idx = (h >> 8) & (PTS - 1);
            Affine<Fq> p;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = pts[idx * 6 + k], ya = pts[idx * 6 + 3 + k];
                p.x.v[4 * k] = xa.x, p.x.v[4 * k + 1] = xa.y, p.x.v[4 * k + 2] = xa.z, p.x.v[4 * k + 3] = xa.w;
                p.y.v[4 * k] = ya.x, p.y.v[4 * k + 1] = ya.y, p.y.v[4 * k + 2] = ya.z, p.y.v[4 * k + 3] = ya.w;
            }
            const Affine<Fq> q = (h & 1) ? aff_neg(p) : p;
            bool done = false;
            if (e == 1 && !acc.is_inf() && !q.is_inf()) done = jac_mmadd(acc, q, acc);
            if (!done) acc = jac_madd(acc, q);
        }
        store_jac<Fq>(partials, (size_t)tid * chunks_per_thread + ch, acc);
    }
    clk_end(rec, c0, w0);
}

// k_accumulate_r28's arithmetic (round 5: unsaturated radix-2^28 Fq, mbls_fq28.hpp): the same
// madd / mmadd with acc.y parked in a per-lane LDS slot across the addition's middle (the kernel
// parks it in its free stage slot), same launch bounds
struct ParkLds {
    uint4* q;  // this lane's 4 pieces, stride 256
    r28::F28 x;
    MBLS_DEV void put(int s, const r28::F28& a) {
        if (s == 0) {
            x = a;
            return;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            q[256 * k] = make_uint4(a.l[4 * k], a.l[4 * k + 1], k < 3 ? a.l[4 * k + 2] : 0u, k < 3 ? a.l[4 * k + 3] : 0u);
        asm volatile("" ::: "memory");
    }
    MBLS_DEV r28::F28 get(int s) const {
        if (s == 0) return x;
        asm volatile("" ::: "memory");
        r28::F28 r;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 u = q[256 * k];
            r.l[4 * k] = u.x;
            r.l[4 * k + 1] = u.y;
            if (k < 3) {
                r.l[4 * k + 2] = u.z;
                r.l[4 * k + 3] = u.w;
            }
        }
        return r;
    }
};

template <int CHUNK>
__global__ __launch_bounds__(256, 3) void k_acc28_ceiling(const uint8_t* __restrict__ table, uint8_t* __restrict__ partials,
                                                          Clk* rec, uint32_t chunks_per_thread, uint32_t seed) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 pts[PTS * 6];
    __shared__ uint4 park[4 * 256];
    for (int k = threadIdx.x; k < PTS * 6; k += blockDim.x) pts[k] = reinterpret_cast<const uint4*>(table)[k];
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = seed ^ (tid * 0x9e3779b9u);
    for (uint32_t ch = 0; ch < chunks_per_thread; ++ch) {
        r28::J28 acc = r28::J28::inf();
        for (int e = 0; e < CHUNK; ++e) {
            h = h * 1664525u + 1013904223u;
            const uint32_t idx = (h >> 8) & (PTS - 1);
            uint32_t xw[12], yw[12];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = pts[idx * 6 + k], ya = pts[idx * 6 + 3 + k];
                xw[4 * k] = xa.x, xw[4 * k + 1] = xa.y, xw[4 * k + 2] = xa.z, xw[4 * k + 3] = xa.w;
                yw[4 * k] = ya.x, yw[4 * k + 1] = ya.y, yw[4 * k + 2] = ya.z, yw[4 * k + 3] = ya.w;
            }
            const r28::F28 qx = r28::unpack_shift8(xw);
            r28::F28 qy = r28::unpack_shift8(yw);
            if (h & 1) qy = r28::neg<r28::B512>(qy);
            bool done = false;
            if (e == 1 && !acc.is_inf()) done = r28::mmadd(acc, qx, qy);
            ParkLds pk{&park[threadIdx.x]};
            if (!done) r28::madd(acc, qx, qy, pk);
        }
        Jacobian<Fq> out;
        r28::to_words(acc.x, out.x.v);
        r28::to_words(acc.y, out.y.v);
        r28::to_words(acc.z, out.z.v);
        store_jac<Fq>(partials, (size_t)tid * chunks_per_thread + ch, out);
    }
    clk_end(rec, c0, w0);
}

// the shipped G1 accumulation's arithmetic since round 6: XYZZ (r28::xmadd / xmmadd, y parked in
// LDS), partials stored as 4 canonical coordinates (192 B)
template <int CHUNK>
__global__ __launch_bounds__(256, 3) void k_acc28x_ceiling(const uint8_t* __restrict__ table, uint8_t* __restrict__ partials,
                                                           Clk* rec, uint32_t chunks_per_thread, uint32_t seed) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 pts[PTS * 6];
    __shared__ uint4 park[4 * 256];
    for (int k = threadIdx.x; k < PTS * 6; k += blockDim.x) pts[k] = reinterpret_cast<const uint4*>(table)[k];
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = seed ^ (tid * 0x9e3779b9u);
    for (uint32_t ch = 0; ch < chunks_per_thread; ++ch) {
        r28::X28 acc = r28::X28::inf();
        for (int e = 0; e < CHUNK; ++e) {
            h = h * 1664525u + 1013904223u;
            const uint32_t idx = (h >> 8) & (PTS - 1);
            uint32_t xw[12], yw[12];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = pts[idx * 6 + k], ya = pts[idx * 6 + 3 + k];
                xw[4 * k] = xa.x, xw[4 * k + 1] = xa.y, xw[4 * k + 2] = xa.z, xw[4 * k + 3] = xa.w;
                yw[4 * k] = ya.x, yw[4 * k + 1] = ya.y, yw[4 * k + 2] = ya.z, yw[4 * k + 3] = ya.w;
            }
            const r28::F28 qx = r28::unpack_shift8(xw);
            r28::F28 qy = r28::unpack_shift8(yw);
            if (h & 1) qy = r28::neg<r28::B512>(qy);
            bool done = false;
            if (e == 1 && !acc.is_inf()) done = r28::xmmadd(acc, qx, qy);
            ParkLds pk{&park[threadIdx.x]};
            if (!done) r28::xmadd(acc, qx, qy, pk);
        }
        uint4* q = reinterpret_cast<uint4*>(partials + ((size_t)tid * chunks_per_thread + ch) * 192);
        auto put = [&](int k, const r28::F28& c) {
            uint32_t w[12];
            r28::to_words(c, w);
#pragma unroll
            for (int j = 0; j < 3; ++j) q[3 * k + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
        };
        put(0, acc.x);
        put(1, acc.y);
        put(2, acc.zz);
        put(3, acc.zzz);
    }
    clk_end(rec, c0, w0);
}

// G2 (round 6): pair-sliced radix-2^28 Fq2, lane j of a pair holding component j; the table holds
// 64 G2 points (192 B: x0 x1 y0 y1), each lane reading its component's words
#ifndef MBLS_ACC_G2_MINW
#define MBLS_ACC_G2_MINW 2
#endif
template <int CHUNK>
__global__ __launch_bounds__(256, MBLS_ACC_G2_MINW) void k_acc28p_ceiling(const uint8_t* __restrict__ table,
                                                                          uint8_t* __restrict__ partials, Clk* rec,
                                                                          uint32_t chunks_per_pair, uint32_t seed) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 pts[PTS * 12];
    for (int k = threadIdx.x; k < PTS * 12; k += blockDim.x) pts[k] = reinterpret_cast<const uint4*>(table)[k];
    __syncthreads();
    const uint32_t pair = (blockIdx.x * blockDim.x + threadIdx.x) >> 1, j = threadIdx.x & 1;
    uint32_t h = seed ^ (pair * 0x9e3779b9u);  // pair-uniform stream
    for (uint32_t ch = 0; ch < chunks_per_pair; ++ch) {
        r28p::J28p acc = r28p::J28p::inf();
        for (int e = 0; e < CHUNK; ++e) {
            h = h * 1664525u + 1013904223u;
            const uint32_t idx = (h >> 8) & (PTS - 1);
            uint32_t xw[12], yw[12];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = pts[idx * 12 + 3 * j + k], ya = pts[idx * 12 + 6 + 3 * j + k];
                xw[4 * k] = xa.x, xw[4 * k + 1] = xa.y, xw[4 * k + 2] = xa.z, xw[4 * k + 3] = xa.w;
                yw[4 * k] = ya.x, yw[4 * k + 1] = ya.y, yw[4 * k + 2] = ya.z, yw[4 * k + 3] = ya.w;
            }
            const r28::F28 qx = r28::unpack_shift8(xw);
            r28::F28 qy = r28::unpack_shift8(yw);
            if (h & 1) qy = r28::carry(r28::neg<r28::B512>(qy));
            if (acc.is_inf()) {
                acc = {r28::fold(qx), r28::fold(qy), r28p::one()};
                continue;
            }
            bool done = false;
            if (e == 1) done = r28p::mmadd(acc, qx, qy);
            if (!done) done = r28p::madd(acc, qx, qy);
            if (!done) acc = r28p::J28p::inf();  // (never for the random table)
        }
        Jacobian<PFq2> out{r28p::to_pf(acc.x), r28p::to_pf(acc.y), r28p::to_pf(acc.z)};
        store_jac<PFq2>(partials, (size_t)pair * chunks_per_pair + ch, out);
    }
    clk_end(rec, c0, w0);
}

// the shipped G2 accumulation since round 6: pair-sliced XYZZ (r28p::xmadd / xmmadd), raw partials
template <int CHUNK>
__global__ __launch_bounds__(256, MBLS_ACC_G2_MINW) void k_acc28px_ceiling(const uint8_t* __restrict__ table,
                                                                          uint8_t* __restrict__ partials, Clk* rec,
                                                                          uint32_t chunks_per_pair, uint32_t seed) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 pts[PTS * 12];
    for (int k = threadIdx.x; k < PTS * 12; k += blockDim.x) pts[k] = reinterpret_cast<const uint4*>(table)[k];
    __syncthreads();
    const uint32_t pair = (blockIdx.x * blockDim.x + threadIdx.x) >> 1, j = threadIdx.x & 1;
    uint32_t h = seed ^ (pair * 0x9e3779b9u);  // pair-uniform stream
    for (uint32_t ch = 0; ch < chunks_per_pair; ++ch) {
        r28p::X28p acc = r28p::X28p::inf();
        for (int e = 0; e < CHUNK; ++e) {
            h = h * 1664525u + 1013904223u;
            const uint32_t idx = (h >> 8) & (PTS - 1);
            uint32_t xw[12], yw[12];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 xa = pts[idx * 12 + 3 * j + k], ya = pts[idx * 12 + 6 + 3 * j + k];
                xw[4 * k] = xa.x, xw[4 * k + 1] = xa.y, xw[4 * k + 2] = xa.z, xw[4 * k + 3] = xa.w;
                yw[4 * k] = ya.x, yw[4 * k + 1] = ya.y, yw[4 * k + 2] = ya.z, yw[4 * k + 3] = ya.w;
            }
            const r28::F28 qx = r28::unpack_shift8(xw);
            r28::F28 qy = r28::unpack_shift8(yw);
            if (h & 1) qy = r28::carry(r28::neg<r28::B512>(qy));
            bool done = false;
            if (e == 1 && !acc.is_inf()) done = r28p::xmmadd(acc, qx, qy);
            if (!done) r28p::xmadd(acc, qx, qy);
        }
        // raw limbs, as k_accumulate_r28p stores its XYZZ partials (store_xyzz28p)
        uint4* q = reinterpret_cast<uint4*>(partials + ((size_t)pair * chunks_per_pair + ch) * 448 + 224 * j);
        uint32_t w[56];
#pragma unroll
        for (int i = 0; i < 14; ++i) {
            w[i] = acc.x.l[i];
            w[14 + i] = acc.y.l[i];
            w[28 + i] = acc.zz.l[i];
            w[42 + i] = acc.zzz.l[i];
        }
#pragma unroll
        for (int k = 0; k < 14; ++k) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
    }
    clk_end(rec, c0, w0);
}

// --------------------------------------------------------------------- k_ntt_pass body ceiling
__constant__ uint32_t TWO_R[8] = {0x00000002u, 0xfffffffeu, 0xfffcb7fdu, 0xa77b4805u,
                                  0x1343b00au, 0x6673b010u, 0x533afa90u, 0xe7db4ea6u};
MBLS_DEV Fr add2r(const Fr& a, const Fr& b) {
    Fr s, d;
    unsigned c = 0, br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
#pragma unroll
    for (int i = 0; i < 8; ++i) d.v[i] = __builtin_subc(s.v[i], TWO_R[i], br, &br);
    const bool keep = !c && br;
#pragma unroll
    for (int i = 0; i < 8; ++i) s.v[i] = keep ? s.v[i] : d.v[i];
    return s;
}
MBLS_DEV Fr sub2r(const Fr& a, const Fr& b) {
    Fr d;
    unsigned br = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
    const uint32_t mask = 0u - br;
#pragma unroll
    for (int i = 0; i < 8; ++i) d.v[i] = __builtin_addc(d.v[i], TWO_R[i] & mask, c, &c);
    return d;
}

__global__ __launch_bounds__(256) void k_ntt_ceiling(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, Clk* rec,
                                                     int iters) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 tw[256 * 2];  // 256 Fr twiddles
    for (int k = threadIdx.x; k < 512; k += blockDim.x) tw[k] = reinterpret_cast<const uint4*>(in)[k];
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fr x0 = load<FrCfg>(in + 32 * ((tid + 1) & 255)), x1 = load<FrCfg>(in + 32 * ((tid + 2) & 255)),
       x2 = load<FrCfg>(in + 32 * ((tid + 3) & 255)), x3 = load<FrCfg>(in + 32 * ((tid + 4) & 255));
    for (int i = 0; i < iters; ++i) {
        const uint32_t j = (tid + 3u * i) & 127u;
        const Fr w1 = load<FrCfg>(&tw[2 * j]), w2 = load<FrCfg>(&tw[2 * (j + 64)]), w3 = load<FrCfg>(&tw[2 * (j + 128)]);
        x1 = fips::mul<FrCfg, false>(x1, w1);
        x3 = fips::mul<FrCfg, false>(x3, w1);
        Fr y0 = add2r(x0, x1), y1 = sub2r(x0, x1), y2 = add2r(x2, x3), y3 = sub2r(x2, x3);
        y2 = fips::mul<FrCfg, false>(y2, w2);
        y3 = fips::mul<FrCfg, false>(y3, w3);
        x0 = add2r(y0, y2);
        x2 = sub2r(y0, y2);
        x1 = add2r(y1, y3);
        x3 = sub2r(y1, y3);
    }
    store<FrCfg>(out + 128 * (size_t)tid, x0);
    store<FrCfg>(out + 128 * (size_t)tid + 32, x1);
    store<FrCfg>(out + 128 * (size_t)tid + 64, x2);
    store<FrCfg>(out + 128 * (size_t)tid + 96, x3);
    clk_end(rec, c0, w0);
}

// the shipped body (round 6): products in radix 2^29 against limb-plane twiddles (ntt.hip)
__global__ __launch_bounds__(256, 5) void k_ntt29_ceiling(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                          Clk* rec, int iters) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 twa[256], twb[256];  // 256 twiddles: limbs 0-3, 4-7
    __shared__ uint32_t twc[256];         // limb 8
    for (int k = threadIdx.x; k < 256; k += blockDim.x) {
        const r29::F29 t = r29::unpack(load<FrCfg>(in + 32 * k));
        twa[k] = make_uint4(t.l[0], t.l[1], t.l[2], t.l[3]);
        twb[k] = make_uint4(t.l[4], t.l[5], t.l[6], t.l[7]);
        twc[k] = t.l[8];
    }
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fr x0 = load<FrCfg>(in + 32 * ((tid + 1) & 255)), x1 = load<FrCfg>(in + 32 * ((tid + 2) & 255)),
       x2 = load<FrCfg>(in + 32 * ((tid + 3) & 255)), x3 = load<FrCfg>(in + 32 * ((tid + 4) & 255));
    auto ldw = [&](uint32_t g) {
        const uint4 a = twa[g], b = twb[g];
        return r29::F29{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, twc[g]}};
    };
    for (int i = 0; i < iters; ++i) {
        const uint32_t j = (tid + 3u * i) & 127u;
        const r29::F29 w1 = ldw(j), w2 = ldw(j + 64), w3 = ldw(j + 128);
        x1 = r29::mul_words(x1, w1);
        x3 = r29::mul_words(x3, w1);
        Fr y0 = add2r(x0, x1), y1 = sub2r(x0, x1), y2 = add2r(x2, x3), y3 = sub2r(x2, x3);
        y2 = r29::mul_words(y2, w2);
        y3 = r29::mul_words(y3, w3);
        x0 = add2r(y0, y2);
        x2 = sub2r(y0, y2);
        x1 = add2r(y1, y3);
        x3 = sub2r(y1, y3);
    }
    store<FrCfg>(out + 128 * (size_t)tid, x0);
    store<FrCfg>(out + 128 * (size_t)tid + 32, x1);
    store<FrCfg>(out + 128 * (size_t)tid + 64, x2);
    store<FrCfg>(out + 128 * (size_t)tid + 96, x3);
    clk_end(rec, c0, w0);
}

// round 6: the same body with each butterfly's two independent products interleaved
// (r29::mul_words2x: their mad chains alternate inside the asm statements)
template <int MINW>
__global__ __launch_bounds__(256, MINW) void k_ntt29x_ceiling(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                              Clk* rec, int iters) {
    unsigned long long c0, w0;
    clk_begin(c0, w0);
    __shared__ uint4 twa[256], twb[256];
    __shared__ uint32_t twc[256];
    for (int k = threadIdx.x; k < 256; k += blockDim.x) {
        const r29::F29 t = r29::unpack(load<FrCfg>(in + 32 * k));
        twa[k] = make_uint4(t.l[0], t.l[1], t.l[2], t.l[3]);
        twb[k] = make_uint4(t.l[4], t.l[5], t.l[6], t.l[7]);
        twc[k] = t.l[8];
    }
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    Fr x0 = load<FrCfg>(in + 32 * ((tid + 1) & 255)), x1 = load<FrCfg>(in + 32 * ((tid + 2) & 255)),
       x2 = load<FrCfg>(in + 32 * ((tid + 3) & 255)), x3 = load<FrCfg>(in + 32 * ((tid + 4) & 255));
    auto ldw = [&](uint32_t g) {
        const uint4 a = twa[g], b = twb[g];
        return r29::F29{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, twc[g]}};
    };
    for (int i = 0; i < iters; ++i) {
        const uint32_t j = (tid + 3u * i) & 127u;
        const r29::F29 w1 = ldw(j), w2 = ldw(j + 64), w3 = ldw(j + 128);
        r29::mul_words2x(x1, w1, x3, w1);
        Fr y0 = add2r(x0, x1), y1 = sub2r(x0, x1), y2 = add2r(x2, x3), y3 = sub2r(x2, x3);
        r29::mul_words2x(y2, w2, y3, w3);
        x0 = add2r(y0, y2);
        x2 = sub2r(y0, y2);
        x1 = add2r(y1, y3);
        x3 = sub2r(y1, y3);
    }
    store<FrCfg>(out + 128 * (size_t)tid, x0);
    store<FrCfg>(out + 128 * (size_t)tid + 32, x1);
    store<FrCfg>(out + 128 * (size_t)tid + 64, x2);
    store<FrCfg>(out + 128 * (size_t)tid + 96, x3);
    clk_end(rec, c0, w0);
}

// ------------------------------------------------------------------------------------ host
struct Timing {
    double ms, mhz_med, mhz_min, mhz_max, wave_cycles_med;
};

static double wall_khz() {
    int dev = 0, khz = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    return khz;
}

template <class Launch>
static Timing run(Launch launch, Clk* d_rec, size_t waves, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();  // warmup
    CK(hipDeviceSynchronize());
    std::vector<float> ms(reps);
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms[r], a, b));
    }
    std::sort(ms.begin(), ms.end());
    std::vector<Clk> rec(waves);
    CK(hipMemcpy(rec.data(), d_rec, waves * sizeof(Clk), hipMemcpyDeviceToHost));
    const double wk = wall_khz();
    std::vector<double> mhz, cyc;
    for (const Clk& c : rec) {
        const double dw = (double)(c.w1 - c.w0), dc = (double)(c.c1 - c.c0);
        if (dw > 100) mhz.push_back(dc / dw * wk / 1e3);
        cyc.push_back(dc);
    }
    std::sort(mhz.begin(), mhz.end());
    std::sort(cyc.begin(), cyc.end());
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return Timing{ms[reps / 2], mhz.empty() ? 0 : mhz[mhz.size() / 2], mhz.empty() ? 0 : mhz.front(),
                  mhz.empty() ? 0 : mhz.back(), cyc[cyc.size() / 2]};
}

int main(int argc, char** argv) {
    const int clog = argc > 1 ? atoi(argv[1]) : 24;  // contributions of the accumulation ceiling
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const double simds = 4.0 * cus;
    // 3 waves per SIMD, 256-thread blocks: one full round of resident waves = cus * 3 blocks
    const int blocks_round = cus * 3;
    Clk* d_rec;
    const size_t max_waves = (size_t)1 << 20;
    CK(hipMalloc(&d_rec, max_waves * sizeof(Clk)));
    uint64_t* d_out;
    CK(hipMalloc(&d_out, (size_t)blocks_round * 16 * 256 * 8));

    printf("{\"device\": \"%s\", \"cus\": %d, \"wall_clock_khz\": %.0f", prop.gcnArchName, cus, wall_khz());
    // ISA rates: 16 rounds of resident waves, 8 independent chains per lane
    const int ib = blocks_round * 16, iters = 4096;
    const char* names[3] = {"v_mad_u64_u32", "v_add_co+v_addc_co (2 instr)", "fips_pair mad+addc (2 instr)"};
    for (int op = 0; op < 3; ++op) {
        auto L = [&] {
            if (op == 0) hipLaunchKernelGGL(k_isa<0>, dim3(ib), dim3(256), 0, 0, d_out, d_rec, 7u, iters);
            if (op == 1) hipLaunchKernelGGL(k_isa<1>, dim3(ib), dim3(256), 0, 0, d_out, d_rec, 7u, iters);
            if (op == 2) hipLaunchKernelGGL(k_isa<2>, dim3(ib), dim3(256), 0, 0, d_out, d_rec, 7u, iters);
        };
        Timing t = run(L, d_rec, (size_t)ib * 4, 5);
        const double wave_instr = (double)ib * 4 * iters * 8 * (op == 0 ? 1 : 2);
        const double simd_cycles = t.ms * 1e-3 * t.mhz_med * 1e6 * simds;
        printf(",\n \"isa_%d\": {\"what\": \"%s\", \"ms\": %.4f, \"mhz_med\": %.0f, \"mhz_min\": %.0f, \"mhz_max\": %.0f, "
               "\"simd_cycles_per_wave_instr\": %.3f, \"lane_ops_per_s_T\": %.3f}",
               op, names[op], t.ms, t.mhz_med, t.mhz_min, t.mhz_max, simd_cycles / wave_instr,
               wave_instr * 64 / (t.ms * 1e-3) / 1e12);
    }
    // accumulation ceiling: 2^clog contributions in 16-point chunks, one partial per chunk
    {
        const size_t contributions = (size_t)1 << clog, chunks = contributions / 16;
        const uint32_t threads = blocks_round * 256 * 4;  // 4 rounds of resident waves
        const uint32_t per = (uint32_t)((chunks + threads - 1) / threads);
        std::vector<uint32_t> tab(PTS * 24);
        uint32_t s = 12345;
        for (auto& w : tab) w = (s = s * 1103515245u + 12345u);
        for (int i = 0; i < PTS * 2; ++i) tab[i * 12 + 11] &= 0x0fffffffu;  // < p
        uint8_t *d_tab, *d_part;
        CK(hipMalloc(&d_tab, tab.size() * 4));
        CK(hipMemcpy(d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_part, (size_t)threads * per * 144));
        auto L = [&] {
            hipLaunchKernelGGL(k_acc_ceiling<16>, dim3(threads / 256), dim3(256), 0, 0, d_tab, d_part, d_rec, per, 99u);
        };
        Timing t = run(L, d_rec, threads / 64, 5);
        const double done = (double)threads * per * 16;
        printf(",\n \"acc_ceiling\": {\"kernel\": \"k_acc_ceiling<16> (k_accumulate<G1> arithmetic, points from LDS)\", "
               "\"contributions\": %.0f, \"ms\": %.4f, \"ns_per_contribution_chip\": %.6f, \"mhz_med\": %.0f, "
               "\"mhz_min\": %.0f, \"mhz_max\": %.0f, \"ms_per_2^20_g1_msm_contributions\": %.4f}",
               done, t.ms, t.ms * 1e6 / done, t.mhz_med, t.mhz_min, t.mhz_max, t.ms / done * 16777216.0);
        auto L28 = [&] {
            hipLaunchKernelGGL(k_acc28_ceiling<16>, dim3(threads / 256), dim3(256), 0, 0, d_tab, d_part, d_rec, per, 99u);
        };
        Timing t28 = run(L28, d_rec, threads / 64, 5);
        printf(",\n \"acc28_ceiling\": {\"kernel\": \"k_acc28_ceiling<16> (k_accumulate_r28 arithmetic: radix-2^28 Fq, "
               "acc.y parked in LDS; points from LDS)\", "
               "\"contributions\": %.0f, \"ms\": %.4f, \"ns_per_contribution_chip\": %.6f, \"mhz_med\": %.0f, "
               "\"mhz_min\": %.0f, \"mhz_max\": %.0f, \"ms_per_2^20_g1_msm_contributions\": %.4f}",
               done, t28.ms, t28.ms * 1e6 / done, t28.mhz_med, t28.mhz_min, t28.mhz_max, t28.ms / done * 16777216.0);
        uint8_t* d_part_x;
        CK(hipMalloc(&d_part_x, (size_t)threads * per * 192));
        auto L28x = [&] {
            hipLaunchKernelGGL(k_acc28x_ceiling<16>, dim3(threads / 256), dim3(256), 0, 0, d_tab, d_part_x, d_rec, per, 99u);
        };
        Timing t28x = run(L28x, d_rec, threads / 64, 5);
        CK(hipFree(d_part_x));
        printf(",\n \"acc28x_ceiling\": {\"kernel\": \"k_acc28x_ceiling<16> (k_accumulate_r28 arithmetic since round 6: "
               "XYZZ madd-2008-s in radix-2^28 Fq, y parked in LDS; points from LDS)\", "
               "\"contributions\": %.0f, \"ms\": %.4f, \"ns_per_contribution_chip\": %.6f, \"mhz_med\": %.0f, "
               "\"mhz_min\": %.0f, \"mhz_max\": %.0f, \"ms_per_2^20_g1_msm_contributions\": %.4f}",
               done, t28x.ms, t28x.ms * 1e6 / done, t28x.mhz_med, t28x.mhz_min, t28x.mhz_max, t28x.ms / done * 16777216.0);
        // G2 pair-sliced: 2^(clog - 2) contributions (a G2 contribution costs ~3x a G1 one)
        {
            const size_t c2 = contributions / 4, chunks2 = c2 / 16;
            const uint32_t pairs = threads / 2;
            const uint32_t per2 = (uint32_t)((chunks2 + pairs - 1) / pairs);
            std::vector<uint32_t> tab2(PTS * 48);
            for (auto& w : tab2) w = (s = s * 1103515245u + 12345u);
            for (int i = 0; i < PTS * 4; ++i) tab2[i * 12 + 11] &= 0x0fffffffu;  // < p
            uint8_t *d_tab2, *d_part2;
            CK(hipMalloc(&d_tab2, tab2.size() * 4));
            CK(hipMemcpy(d_tab2, tab2.data(), tab2.size() * 4, hipMemcpyHostToDevice));
            CK(hipMalloc(&d_part2, (size_t)pairs * per2 * 288));
            auto LG2 = [&] {
                hipLaunchKernelGGL(k_acc28p_ceiling<16>, dim3(threads / 256), dim3(256), 0, 0, d_tab2, d_part2, d_rec, per2, 77u);
            };
            Timing tg = run(LG2, d_rec, threads / 64, 5);
            const double done2 = (double)pairs * per2 * 16;
            // G2 2^20 MSM: psi split, 4n digit streams x 4 windows of c = 16
            printf(",\n \"acc28p_ceiling\": {\"kernel\": \"k_acc28p_ceiling<16> (k_accumulate_r28p<G2> arithmetic: "
                   "pair-sliced radix-2^28 Fq2; points from LDS)\", \"contributions\": %.0f, \"ms\": %.4f, "
                   "\"ns_per_contribution_chip\": %.6f, \"mhz_med\": %.0f, \"ms_per_2^20_g2_msm_contributions\": %.4f}",
                   done2, tg.ms, tg.ms * 1e6 / done2, tg.mhz_med, tg.ms / done2 * 16777216.0);
            uint8_t* d_part2x;
            CK(hipMalloc(&d_part2x, (size_t)pairs * per2 * 448));
            auto LG2x = [&] {
                hipLaunchKernelGGL(k_acc28px_ceiling<16>, dim3(threads / 256), dim3(256), 0, 0, d_tab2, d_part2x, d_rec, per2, 77u);
            };
            Timing tgx = run(LG2x, d_rec, threads / 64, 5);
            printf(",\n \"acc28px_ceiling\": {\"kernel\": \"k_acc28px_ceiling<16> (k_accumulate_r28p<G2> arithmetic since round 6: "
                   "pair-sliced radix-2^28 XYZZ; points from LDS)\", \"contributions\": %.0f, \"ms\": %.4f, "
                   "\"ns_per_contribution_chip\": %.6f, \"mhz_med\": %.0f, \"ms_per_2^20_g2_msm_contributions\": %.4f}",
                   done2, tgx.ms, tgx.ms * 1e6 / done2, tgx.mhz_med, tgx.ms / done2 * 16777216.0);
            CK(hipFree(d_part2x));
            CK(hipFree(d_tab2));
            CK(hipFree(d_part2));
        }
        CK(hipFree(d_tab));
        CK(hipFree(d_part));
    }
    // NTT radix-4 body ceiling
    {
        const int nb = blocks_round * 8 / 3 * 5;  // ~5 waves per SIMD (LDS-bound occupancy of the pass)
        const int it = 512;
        uint8_t *d_in, *d_o;
        std::vector<uint32_t> v(256 * 8);
        uint32_t s = 777;
        for (auto& w : v) w = (s = s * 1103515245u + 12345u);
        for (int i = 0; i < 256; ++i) v[i * 8 + 7] &= 0x3fffffffu;  // < r
        CK(hipMalloc(&d_in, v.size() * 4));
        CK(hipMemcpy(d_in, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        CK(hipMalloc(&d_o, (size_t)nb * 256 * 128));
        auto L = [&] { hipLaunchKernelGGL(k_ntt_ceiling, dim3(nb), dim3(256), 0, 0, d_in, d_o, d_rec, it); };
        Timing t = run(L, d_rec, (size_t)nb * 4, 5);
        const double bf = (double)nb * 256 * it;  // radix-4 butterflies (2 stages x 4 elements each)
        // one 2^22 transform: 11 stage pairs x 2^20 radix-4 butterflies, the first pair without products
        printf(",\n \"ntt_ceiling\": {\"kernel\": \"k_ntt_ceiling (k_ntt_pass radix-4 body, twiddles from LDS)\", "
               "\"radix4_butterflies\": %.0f, \"ms\": %.4f, \"G_radix4_per_s\": %.3f, \"mhz_med\": %.0f, "
               "\"ms_per_2^22_transform_10_pairs\": %.4f}",
               bf, t.ms, bf / (t.ms * 1e-3) / 1e9, t.mhz_med, 10.0 * (1 << 20) / (bf / (t.ms * 1e-3)) * 1e3);
        auto L29 = [&] { hipLaunchKernelGGL(k_ntt29_ceiling, dim3(nb), dim3(256), 0, 0, d_in, d_o, d_rec, it); };
        Timing t29 = run(L29, d_rec, (size_t)nb * 4, 5);
        printf(",\n \"ntt29_ceiling\": {\"kernel\": \"k_ntt29_ceiling (the shipped k_ntt_pass radix-4 body: radix-2^29 "
               "products, twiddle limb planes from LDS)\", \"radix4_butterflies\": %.0f, \"ms\": %.4f, "
               "\"G_radix4_per_s\": %.3f, \"mhz_med\": %.0f, \"ms_per_2^22_transform_10_pairs\": %.4f}",
               bf, t29.ms, bf / (t29.ms * 1e-3) / 1e9, t29.mhz_med, 10.0 * (1 << 20) / (bf / (t29.ms * 1e-3)) * 1e3);
        for (int mw = 5; mw >= 4; --mw) {
            auto L29x = [&] {
                if (mw == 5)
                    hipLaunchKernelGGL(k_ntt29x_ceiling<5>, dim3(nb), dim3(256), 0, 0, d_in, d_o, d_rec, it);
                else
                    hipLaunchKernelGGL(k_ntt29x_ceiling<4>, dim3(nb), dim3(256), 0, 0, d_in, d_o, d_rec, it);
            };
            Timing t29x = run(L29x, d_rec, (size_t)nb * 4, 5);
            printf(",\n \"ntt29x%d_ceiling\": {\"kernel\": \"k_ntt29x_ceiling<%d> (the radix-4 body with each butterfly's two "
                   "independent products interleaved, r29::mul_words2x; %d waves per SIMD)\", \"radix4_butterflies\": %.0f, \"ms\": %.4f, "
                   "\"G_radix4_per_s\": %.3f, \"mhz_med\": %.0f, \"ms_per_2^22_transform_10_pairs\": %.4f}",
                   mw, mw, mw, bf, t29x.ms, bf / (t29x.ms * 1e-3) / 1e9, t29x.mhz_med, 10.0 * (1 << 20) / (bf / (t29x.ms * 1e-3)) * 1e3);
        }
        CK(hipFree(d_in));
        CK(hipFree(d_o));
    }
    printf("\n}\n");
    CK(hipFree(d_rec));
    CK(hipFree(d_out));
    return 0;
}
