// mbls_fr29.hpp -- BLS12-381 Fr products in unsaturated radix 2^29 for the NTT butterflies.
//
// Why: on gfx950 every wave64 VALU instruction issues over ~4 SIMD cycles, v_mad_u64_u32 as much as
// v_addc_co_u32 (tools/valu_ceiling.hip).  The 32-bit product-scanning Montgomery product
// (mbls_fips.hpp) pays one v_addc for the column-overflow counter after every v_mad_u64_u32 and
// two v_mov per column shift: ~290 instructions per Fr product, 128 of them carries.  With 9 limbs
// of 29 bits a partial product is < 2^58 and a column of <= 9 products plus <= 8 reduction terms
// stays below 2^64, so every column is a plain v_mad_u64_u32 chain into one 64-bit accumulator
// shifted by one v_lshrrev_b64: 81 product + 72 reduction mads and ~50 other instructions.  With
// the 32 instructions that split the multiplicand into limbs and pack the product back into
// words, a twiddle product costs ~240 instructions instead of ~290 (the same trick as the
// radix-2^28 Fq of mbls_fq28.hpp; the NTT keeps its data, its LDS tile and its [0, 2r) lazy
// additions in 32-bit words -- only the products change representation).
//
// Representation.  9 limbs l_i, value sum l_i 2^(29 i).  Montgomery radix R' = 2^261: the
// product is a b / 2^261 mod r.  Data stay x R mod r (R = 2^256, the library's format); the
// twiddle tables hold w R' mod r (k_twiddles), so mul(x R, w R') = x w R: the products land in
// the data's own Montgomery form with no conversion.
//
// Bounds (tests/test_gpu_limbs.py drives them at the extremes, bit-exact against Python integers):
//   * column k: <= 9 products a_i b_j + <= 8 terms m_i r_j (< 2^58) + m_k (< 2^29) + the carry
//     (< 2^35) < 2^64 needs 9 2^(A+B) < 2^64 - 2^61, i.e. A + B <= 60.6 for limbs a_i < 2^A,
//     b_j < 2^B -- here both operands are normalised (A = B = 29);
//   * output: (a b + m r) / 2^261 < a b / 2^261 + r, normalised limbs (the top one < 2^27 for
//     the outputs below); for a < 2^256 (any word operand) and b < r: < r (1 + 2^256 / 2^261)
//     < 1.04 r -- in [0, 2r) and below 2^256, so the lazy butterflies take it as words.
#pragma once
#include "mbls_field.hpp"
#include "mbls_madchain.hpp"

namespace mbls {
namespace r29 {

constexpr int NL = 9;
constexpr uint32_t MASK = (1u << 29) - 1;
// r in radix 2^29; r = 1 (mod 2^29), so -r^-1 = -1 (mod 2^29): m_k = -acc mod 2^29 and m_k r_0 = m_k
constexpr uint32_t RL[NL] = {0x1u,        0x1ffffff8u, 0x1f96ffbfu, 0x1b4805ffu, 0x1d80553bu,
                             0x0c0404d0u, 0x1520cce7u, 0x0a6533afu, 0x0073eda7u};
static_assert(RL[0] == 1u, "the reduction relies on r = 1 mod 2^29");

struct F29 {
    uint32_t l[NL];
};

// 8 canonical-or-lazy words (any value < 2^256) -> 9 normalised limbs (value unchanged)
MBLS_DEV F29 unpack(const Fr& a) {
    F29 r;
    r.l[0] = a.v[0] & MASK;
#pragma unroll
    for (int i = 1; i < NL; ++i) {
        const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
        const uint32_t lo = a.v[wi], hi = wi + 1 < 8 ? a.v[wi + 1] : 0u;
        const uint32_t v = sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo;
        r.l[i] = i < NL - 1 ? (v & MASK) : v;  // the top limb holds bits 232..255
    }
    return r;
}

// normalised limbs of a value < 2^256 -> 8 words
MBLS_DEV Fr pack(const F29& a) {
    Fr r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        // bits [32 j, 32 j + 32): limb k = floor(32 j / 29) from bit s, then limb k + 1 (and k + 2)
        const int k = (32 * j) / 29, s = (32 * j) % 29;
        uint32_t w = a.l[k] >> s;
        if (k + 1 < NL) w |= a.l[k + 1] << (29 - s);
        if (k + 2 < NL && 58 - s < 32) w |= a.l[k + 2] << (58 - s);
        r.v[j] = w;
    }
    return r;
}

// Montgomery product a b / 2^261 (lazy: no final subtraction), product scanning; column k
// accumulates its a_i b_(k-i) and m_i r_(k-i) in ONE 64-bit register, one v_mad_u64_u32 chain
// (mbls_madchain.hpp: written as C++ additions LLVM splits every column into a fresh chain plus a
// 64-bit merge add).  Columns by compile-time recursion.
template <int K>
MBLS_DEV void mul_cols(uint64_t& acc, uint32_t (&m)[NL], F29& r, const F29& a, const F29& b) {
    if constexpr (K < 2 * NL - 1) {
        constexpr int LO = K > NL - 1 ? K - (NL - 1) : 0;
        madc::col<K, LO, (K < NL - 1 ? K : NL - 1), false>(acc, a.l, b.l);
        madc::col<K, LO, (K < NL ? K : NL) - 1, true>(acc, m, RL);
        if constexpr (K < NL) {
            m[K] = (0u - (uint32_t)acc) & MASK;
            acc += m[K];  // m_k r_0, r_0 = 1: the low 29 bits become zero
        } else {
            r.l[K - NL] = (uint32_t)acc & MASK;
        }
        acc >>= 29;
        mul_cols<K + 1>(acc, m, r, a, b);
    }
}
MBLS_DEV F29 mul(const F29& a, const F29& b) {
    uint32_t m[NL];
    F29 r;
    uint64_t acc = 0;
    mul_cols<0>(acc, m, r, a, b);
    r.l[NL - 1] = (uint32_t)acc;
    return r;
}

// x w R'^-1 for word data x (< 2^256) and a normalised twiddle limb set w (< r): x w R mod r in
// [0, 2r) as words when x is x R, w is w R' (see the header)
MBLS_DEV Fr mul_words(const Fr& x, const F29& w) { return pack(mul(unpack(x), w)); }

// two independent products a b, c d column by column, their mad chains interleaved
// (madc::col2): the same values as two mul() calls.  Measured in tools/valu_ceiling.hip
// (k_ntt29x_ceiling): no faster than two mul() calls at 4-5 waves per SIMD (the mad latency is
// already hidden), so the NTT pass does not use it (profiles/r06/README.md)
template <int K>
MBLS_DEV void mul2x_cols(uint64_t& p, uint32_t (&m)[NL], F29& r, const F29& a, const F29& b, uint64_t& q,
                         uint32_t (&n)[NL], F29& t, const F29& c, const F29& d) {
    if constexpr (K < 2 * NL - 1) {
        constexpr int LO = K > NL - 1 ? K - (NL - 1) : 0;
        madc::col2<K, LO, (K < NL - 1 ? K : NL - 1), false>(p, a.l, b.l, q, c.l, d.l);
        madc::col2<K, LO, (K < NL ? K : NL) - 1, true>(p, m, RL, q, n, RL);
        if constexpr (K < NL) {
            m[K] = (0u - (uint32_t)p) & MASK;
            n[K] = (0u - (uint32_t)q) & MASK;
            p += m[K];
            q += n[K];
        } else {
            r.l[K - NL] = (uint32_t)p & MASK;
            t.l[K - NL] = (uint32_t)q & MASK;
        }
        p >>= 29;
        q >>= 29;
        mul2x_cols<K + 1>(p, m, r, a, b, q, n, t, c, d);
    }
}
MBLS_DEV void mul2x(F29& r, const F29& a, const F29& b, F29& t, const F29& c, const F29& d) {
    uint32_t m[NL], n[NL];
    uint64_t p = 0, q = 0;
    mul2x_cols<0>(p, m, r, a, b, q, n, t, c, d);
    r.l[NL - 1] = (uint32_t)p;
    t.l[NL - 1] = (uint32_t)q;
}
MBLS_DEV void mul_words2x(Fr& x, const F29& w, Fr& y, const F29& v) {
    F29 r, t;
    mul2x(r, unpack(x), w, t, unpack(y), v);
    x = pack(r);
    y = pack(t);
}

}  // namespace r29
}  // namespace mbls
