// msm_common.hip -- group-independent MSM stages: plan, signed-digit decomposition, scans,
// counting-sort scatter, chunking, synthetic scalars.
//
// Reference: get_optimal_c (msm.cuh:115-133), compute_bucket_indices_kernel
// (msm_kernels.cu:69-143), histogram (:224-256), cub ExclusiveSum / SortPairs (:748-781).
#include <hip/hip_runtime.h>

#include "msm_core.hpp"

namespace mbls {

// window size: the reference's size classes (msm.cuh:115-133) except c = 15, where
// 17 * 15 = 255 leaves an 18th window holding only the final carry -- one bucket with about
// half of all points (measured: 1.3 s of serial bucket summation at 2^20).  c = 16 instead.
static int optimal_c(long long n) {
    if (n <= (1 << 8)) return 7;
    if (n <= (1 << 10)) return 8;
    if (n <= (1 << 12)) return 10;
    if (n <= (1 << 14)) return 12;
    if (n <= (1 << 16)) return 13;
    if (n <= (1 << 18)) return 14;
    return 16;
}

eIcicleError make_plan(long long n, const MSMConfig* cfg, MsmPlan& p) {
    int c = cfg->c > 0 ? cfg->c : optimal_c(n);
    if (c < 2 || c > 20) return MBLS_INVALID_ARGUMENT;
    int bits = cfg->bitsize > 0 ? cfg->bitsize : 255;
    if (bits > 256) return MBLS_INVALID_ARGUMENT;
    // signed digits need one bit of headroom for the top carry
    int W = (bits + 1 + c - 1) / c;
    int F = cfg->precompute_factor > 0 ? cfg->precompute_factor : 1;
    if (F > W) F = W;
    int Wg = (W + F - 1) / F;
    p.c = c;
    p.W = W;
    p.F = F;
    p.Wg = Wg;
    p.B = 1u << (c - 1);
    p.TB = (uint32_t)Wg * p.B;
    p.contributions = (size_t)n * W;
    if ((size_t)n * F >= (1u << 31)) return MBLS_INVALID_ARGUMENT;
    // reduction levels: level 0 has B inputs, each level divides by SEG, the last has 1 output
    p.levels = 0;
    uint32_t m = p.B;
    while (true) {
        if (p.levels >= MAX_LEVELS) return MBLS_INVALID_ARGUMENT;
        p.level_m[p.levels++] = m;
        const uint32_t seg = level_seg(p.levels - 1);
        uint32_t mo = (m + seg - 1) / seg;
        if (mo <= 1) break;
        m = mo;
    }
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 1. digits: one thread per scalar
// ------------------------------------------------------------------------------------
template <bool MONT>
__global__ __launch_bounds__(256) void k_digits(const uint8_t* __restrict__ scalars, uint32_t n, int c, int W, int Wg, uint32_t F,
                                                uint32_t B, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                uint32_t* __restrict__ counts) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = load<FrCfg>(scalars + 32 * (size_t)i);
    if (MONT) s = from_mont(s);
    uint32_t carry = 0;
    const uint32_t mask = (1u << c) - 1;
    for (int w = 0; w < W; ++w) {
        const int bit = w * c;
        const int word = bit >> 5, sh = bit & 31;
        // select words without dynamic register indexing (which would go to scratch)
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            lo = (k == word) ? s.v[k] : lo;
            hi = (k == word + 1) ? s.v[k] : hi;
        }
        uint64_t win = ((uint64_t)hi << 32) | lo;
        uint32_t v = ((uint32_t)(win >> sh) & mask) + carry;
        carry = 0;
        uint32_t sign = 0;
        if (v > B) {  // signed digit: v - 2^c, carry into the next window (msm_kernels.cu:111-117)
            v = (1u << c) - v;
            sign = 1;
            carry = 1;
        }
        const size_t o = (size_t)w * n + i;
        const int f = w / Wg, wl = w % Wg;
        // precomputed bases are point-major: [P_i, 2^l P_i, ..., 2^((F-1) l) P_i] (core/msm.rs:164-165)
        uint32_t key = INVALID_KEY;
        if (v != 0) {
            key = (uint32_t)wl * B + (v - 1);
            vals[o] = ((i * F + (uint32_t)f) << 1) | sign;
        }
        keys[o] = key;
        // histogram: one atomic per wave when the whole wave hits one bucket (adversarial
        // inputs: equal scalars), else one per lane
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
        const uint64_t active = __ballot(1);
        const uint64_t same = __ballot(key == k0);
        if (same == active) {
            if (k0 != INVALID_KEY && __lane_id() == (uint32_t)__builtin_ctzll(active))
                atomicAdd(&counts[k0], (uint32_t)__popcll(active));
        } else if (key != INVALID_KEY) {
            atomicAdd(&counts[key], 1u);
        }
    }
    // canonical scalars (< r < 2^255) never leave a final carry: W*c >= 256 (checked for
    // c = 7..16 in tests/test_oracle.py)
}

eIcicleError launch_digits(const uint8_t* scalars, bool mont, uint32_t n, const MsmPlan& P, uint32_t* keys,
                           uint32_t* vals, uint32_t* counts, hipStream_t st) {
    dim3 g((n + 255) / 256);
    if (mont)
        hipLaunchKernelGGL(k_digits<true>, g, dim3(256), 0, st, scalars, n, P.c, P.W, P.Wg, (uint32_t)P.F, P.B, keys,
                           vals, counts);
    else
        hipLaunchKernelGGL(k_digits<false>, g, dim3(256), 0, st, scalars, n, P.c, P.W, P.Wg, (uint32_t)P.F, P.B, keys,
                           vals, counts);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 2. exclusive scan: three phases, 1024 elements per block, wave64 shuffles
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ void block_scan_1024(uint32_t (&x)[4], uint32_t* sh_wave, uint32_t& total) {
    uint32_t s0 = x[0], s1 = s0 + x[1], s2 = s1 + x[2], s3 = s2 + x[3];
    uint32_t incl = wave_incl_scan(s3);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 63) sh_wave[wid] = incl;
    __syncthreads();
    uint32_t wave_off = 0;
    for (int k = 0; k < wid; ++k) wave_off += sh_wave[k];
    total = sh_wave[0] + sh_wave[1] + sh_wave[2] + sh_wave[3];
    uint32_t excl = wave_off + incl - s3;
    x[0] = excl;
    x[1] = excl + s0;
    x[2] = excl + s1;
    x[3] = excl + s2;
}

__global__ __launch_bounds__(256) void k_scan_local(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    uint32_t* __restrict__ block_sums, uint32_t m) {
    __shared__ uint32_t sh[4];
    uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * 4;
    uint32_t x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = (base + k < m) ? in[base + k] : 0u;
    uint32_t total;
    block_scan_1024(x, sh, total);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < m) out[base + k] = x[k];
    if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_blocks(uint32_t* __restrict__ sums, uint32_t nb, uint32_t* __restrict__ grand) {
    __shared__ uint32_t sh[4];
    uint32_t carry = 0;
    for (uint32_t off = 0; off < nb; off += SCAN_BLOCK) {
        uint32_t base = off + threadIdx.x * 4;
        uint32_t x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = (base + k < nb) ? sums[base + k] : 0u;
        uint32_t total;
        block_scan_1024(x, sh, total);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + k < nb) sums[base + k] = x[k] + carry;
        carry += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) *grand = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* __restrict__ out, const uint32_t* __restrict__ sums, uint32_t m,
                                                  const uint32_t* __restrict__ grand) {
    uint32_t base = blockIdx.x * SCAN_BLOCK + threadIdx.x * 4;
    uint32_t add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < m) out[base + k] += add;
    if (blockIdx.x == 0 && threadIdx.x == 0) out[m] = *grand;
}

size_t scan_tmp_words(uint32_t m) { return (m + SCAN_BLOCK - 1) / SCAN_BLOCK + 8; }

eIcicleError scan_exclusive(const uint32_t* in, uint32_t* out, uint32_t m, uint32_t* tmp, hipStream_t st) {
    uint32_t nb = (m + SCAN_BLOCK - 1) / SCAN_BLOCK;
    hipLaunchKernelGGL(k_scan_local, dim3(nb), dim3(256), 0, st, in, out, tmp, m);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(256), 0, st, tmp, nb, tmp + nb);
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(256), 0, st, out, tmp, m, tmp + nb);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// chunks per bucket; nchunks[m] receives the maximum (drives the heavy-bucket tree passes)
__global__ void k_chunk_counts(const uint32_t* __restrict__ counts, uint32_t* __restrict__ nchunks, uint32_t m) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t c = 0;
    if (b < m) {
        c = (counts[b] + CHUNK - 1) / CHUNK;
        nchunks[b] = c;
    }
    // wave max, one atomic per wave
    for (int d = 32; d > 0; d >>= 1) c = max(c, (uint32_t)__shfl_xor(c, d, 64));
    if ((threadIdx.x & 63) == 0 && c > 1) atomicMax(&nchunks[m], c);
}

eIcicleError launch_chunk_counts(const uint32_t* counts, uint32_t* nchunks, uint32_t m, hipStream_t st) {
    MBLS_TRY(hipMemsetAsync(nchunks + m, 0, 4, st));
    hipLaunchKernelGGL(k_chunk_counts, dim3((m + 255) / 256), dim3(256), 0, st, counts, nchunks, m);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// 3. scatter (counting sort)
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_scatter(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                 size_t total, uint32_t* __restrict__ cursor, uint32_t* __restrict__ sorted) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= total) return;
    const uint32_t k = keys[i];
    // wave-uniform bucket (adversarial inputs): one atomic reserves the wave's slots
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(k);
    const uint64_t active = __ballot(1);
    if (__ballot(k == k0) == active) {
        if (k0 == INVALID_KEY) return;
        uint32_t base = 0;
        const uint32_t leader = (uint32_t)__builtin_ctzll(active);
        if (__lane_id() == leader) base = atomicAdd(&cursor[k0], (uint32_t)__popcll(active));
        base = __shfl(base, leader, 64);
        const uint32_t rank = (uint32_t)__popcll(active & ((1ull << __lane_id()) - 1));
        sorted[base + rank] = vals[i];
        return;
    }
    if (k == INVALID_KEY) return;
    uint32_t pos = atomicAdd(&cursor[k], 1u);
    sorted[pos] = vals[i];
}

eIcicleError launch_scatter(const uint32_t* keys, const uint32_t* vals, size_t total, uint32_t* cursor,
                            uint32_t* sorted, hipStream_t st) {
    hipLaunchKernelGGL(k_scatter, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, keys, vals, total, cursor,
                       sorted);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

__global__ void k_chunk_owner(const uint32_t* __restrict__ chunk_off, uint32_t m, uint32_t* __restrict__ owner) {
    uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= m) return;
    for (uint32_t k = chunk_off[b]; k < chunk_off[b + 1]; ++k) owner[k] = b;
}

eIcicleError launch_chunk_owner(const uint32_t* chunk_off, uint32_t m, uint32_t* owner, hipStream_t st) {
    hipLaunchKernelGGL(k_chunk_owner, dim3((m + 255) / 256), dim3(256), 0, st, chunk_off, m, owner);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

// ------------------------------------------------------------------------------------
// scalars
// ------------------------------------------------------------------------------------
__global__ void k_scalars_from_mont(uint8_t* s, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    store<FrCfg>(s + 32 * i, from_mont(load<FrCfg>(s + 32 * i)));
}

eIcicleError launch_scalars_from_mont(uint8_t* s, size_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_scalars_from_mont, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, s, n);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}

__global__ void k_gen_scalars(uint8_t* out, uint64_t seed, size_t n, int mont) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = gen_scalar(seed, i);
    if (mont) s = to_mont(s);
    store<FrCfg>(out + 32 * i, s);
}

}  // namespace mbls

using namespace mbls;

extern "C" eIcicleError mbls_gen_scalars(mbls_fr_t* out_device, uint64_t seed, size_t n, bool montgomery, void* stream) {
    if (!out_device) return MBLS_INVALID_POINTER;
    if (n == 0) return MBLS_SUCCESS;
    hipLaunchKernelGGL(k_gen_scalars, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (uint8_t*)out_device, seed, n, montgomery ? 1 : 0);
    MBLS_TRY(hipGetLastError());
    return MBLS_SUCCESS;
}
