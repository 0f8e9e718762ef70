// mbls_fips.hpp -- product-scanning (FIPS) Montgomery multiplication and squaring.
//
// Column k of a*b + m*p is accumulated in a 64-bit pair `acc` plus a 32-bit overflow counter:
// every partial product is ONE v_mad_u64_u32 (32x32 + 64 -> 64, carry-out to an SGPR pair)
// followed by ONE v_addc_co_u32 of that carry into the counter -- no v_mov traffic to build
// 64-bit addends, which is what dominates the CIOS formulation on gfx950 (mbls_field.hpp:
// ~1.3 K instructions per Fq product, half of them v_mov / 64-bit adds).
// Squaring computes each cross product a_i a_j (i < j) once and doubles the column.
// Inline asm is used only for the mad+addc pair; hipcc schedules and allocates around it.
#pragma once
#include "mbls_field.hpp"

namespace mbls {
namespace fips {

// acc += a*b, cnt += carry-out  (cnt counts 2^64 overflows of the column)
MBLS_DEV void mac(uint64_t& acc, uint32_t& cnt, uint32_t a, uint32_t b) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "v_addc_co_u32 %2, %1, 0, %2, %1"
        : "+v"(acc), "=&s"(c), "+v"(cnt)
        : "v"(a), "v"(b));
}

// same with a wave-uniform (SGPR) multiplier: modulus words live in SGPRs, not VGPR copies
MBLS_DEV void mac_s(uint64_t& acc, uint32_t& cnt, uint32_t a, uint32_t s) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
        "v_addc_co_u32 %2, %1, 0, %2, %1"
        : "+v"(acc), "=&s"(c), "+v"(cnt)
        : "v"(a), "s"(s));
}

// column shift: (acc, cnt) -> value >> 32
MBLS_DEV void shift(uint64_t& acc, uint32_t& cnt) {
    acc = (acc >> 32) | ((uint64_t)cnt << 32);
    cnt = 0;
}

template <class C>
MBLS_DEV Fp<C> mul(const Fp<C>& a, const Fp<C>& b) {
    constexpr int N = C::N;
    uint32_t m[N];
    Fp<C> r;
    uint64_t acc = 0;
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; ++k) {
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k : N - 1); ++i) mac(acc, cnt, a.v[i], b.v[k - i]);
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); ++i) mac_s(acc, cnt, m[i], C::MOD[k - i]);
        if (k < N) {
            m[k] = (uint32_t)acc * C::NINV;
            mac_s(acc, cnt, m[k], C::MOD[0]);  // low word becomes 0
        } else {
            r.v[k - N] = (uint32_t)acc;
        }
        shift(acc, cnt);
    }
    r.v[N - 1] = (uint32_t)acc;
    reduce_once(r);
    return r;
}

// cross products once, doubled: column k = 2*sum_{i<j, i+j=k} a_i a_j + [k even] a_{k/2}^2
template <class C>
MBLS_DEV Fp<C> sqr(const Fp<C>& a) {
    constexpr int N = C::N;
    uint32_t m[N];
    Fp<C> r;
    uint64_t acc = 0;
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 2 * N - 1; ++k) {
        // cross terms into a separate column accumulator, then double and merge
        uint64_t x = 0;
        uint32_t xc = 0;
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i < k - i; ++i) mac(x, xc, a.v[i], a.v[k - i]);
        // acc += 2 * (x, xc)
        {
            uint64_t x2 = x << 1;
            uint32_t xc2 = (xc << 1) | (uint32_t)(x >> 63);
            uint64_t s = acc + x2;
            cnt += xc2 + (s < acc ? 1u : 0u);
            acc = s;
        }
        if ((k & 1) == 0) mac(acc, cnt, a.v[k / 2], a.v[k / 2]);
#pragma unroll
        for (int i = (k < N ? 0 : k - N + 1); i <= (k < N ? k - 1 : N - 1); ++i) mac_s(acc, cnt, m[i], C::MOD[k - i]);
        if (k < N) {
            m[k] = (uint32_t)acc * C::NINV;
            mac_s(acc, cnt, m[k], C::MOD[0]);
        } else {
            r.v[k - N] = (uint32_t)acc;
        }
        shift(acc, cnt);
    }
    r.v[N - 1] = (uint32_t)acc;
    reduce_once(r);
    return r;
}

}  // namespace fips
}  // namespace mbls
