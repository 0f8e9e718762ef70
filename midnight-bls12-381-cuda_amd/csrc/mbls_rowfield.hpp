// mbls_rowfield.hpp -- "row-sliced" Fq / Fq2 arithmetic for latency-bound serial chains.
//
// Why: on CDNA4 a lone lane needs ~2.5 us per Fq Montgomery product (~1.3 K dependent
// instructions at one wave per SIMD), so a Jacobian addition is ~40 us and the MSM's serial
// phases (bucket-reduction chains, the window Horner of ~240 doublings) dominated the MSM
// (profiles/r01).  Here ONE field element is spread over a 16-lane DPP row: lane j holds
// 32-bit limb j (j < 12), lanes 12..15 hold zero.  A product is a lane-parallel CIOS: per
// word of b one DPP row broadcast, two v_mad_u64_u32 and a DPP row shift (~10 instructions
// per lane per word), and carries are resolved at the end with a carry-lookahead computed on
// the 64-bit ballot masks.  ~150 instructions per lane per product instead of ~1.3 K.
// A wave holds 4 independent elements (4 rows = 4 logical threads).
//
// Row isolation: padding lanes 12..15 are zero and values stay < 2^384, so no carry or
// borrow ever crosses from one row into the next inside the 64-bit masks.
// Requirement: all 16 lanes of a row are active together (rows diverge only as a whole).
#pragma once
#include "mbls_field.hpp"

namespace mbls {

namespace rowdpp {
// DPP controls (gfx9 / gfx90a+): row_newbcast:k = 0x150+k, row_shl:1 = 0x101, row_shr:1 = 0x111
template <int K>
MBLS_DEV uint32_t bcast(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x150 + K, 0xf, 0xf, false);
}
MBLS_DEV uint32_t from_up(uint32_t x) {  // lane j <- lane j+1 (row_shl:1), lane 15 <- 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xf, 0xf, true);
}
MBLS_DEV uint32_t from_down(uint32_t x) {  // lane j <- lane j-1 (row_shr:1), lane 0 <- 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
}
MBLS_DEV uint32_t lane16() { return __lane_id() & 15; }
MBLS_DEV uint32_t row_shift() { return __lane_id() & 48; }  // bit offset of this row in a mask
}  // namespace rowdpp

// carry-in vector of a lane-wise addition with generate G / propagate P masks (G & P == 0):
// bit j = g_{j-1} | (p_{j-1} & c_{j-1})  ==  ((G|P) + G) ^ (G|P) ^ G.
// Propagate bits are restricted to limb lanes (0..11 of each row): padding lanes compare
// equal (0 == 0) and would otherwise carry a borrow across the row boundary.
static constexpr uint64_t RF_LIMB_LANES = 0x0fff0fff0fff0fffull;
MBLS_DEV uint64_t carries_in(uint64_t G, uint64_t P) {
    P &= RF_LIMB_LANES;
    const uint64_t a = G | P;
    return (a + G) ^ a ^ G;
}

struct RFq {
    uint32_t v;  // this lane's limb (lanes 12..15: 0)

    MBLS_DEV static uint32_t mod_limb() {
        const uint32_t j = rowdpp::lane16();
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) m = (j == (uint32_t)k) ? FqCfg::MOD[k] : m;
        return m;
    }
    MBLS_DEV static RFq zero() { return {0u}; }
    MBLS_DEV static RFq one() {
        const uint32_t j = rowdpp::lane16();
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) m = (j == (uint32_t)k) ? FqCfg::ONE[k] : m;
        return {m};
    }
    MBLS_DEV static RFq r2() {
        const uint32_t j = rowdpp::lane16();
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < 12; ++k) m = (j == (uint32_t)k) ? FqCfg::R2[k] : m;
        return {m};
    }
    // row-uniform predicates
    MBLS_DEV bool is_zero() const {
        const uint64_t nz = __ballot(v != 0);
        return ((nz >> rowdpp::row_shift()) & 0xffffull) == 0;
    }
    MBLS_DEV bool operator==(const RFq& o) const {
        const uint64_t ne = __ballot(v != o.v);
        return ((ne >> rowdpp::row_shift()) & 0xffffull) == 0;
    }
};

// canonical r = t - p if t >= p else t   (t < 2p, canonical limbs)
MBLS_DEV RFq rf_reduce_once(uint32_t t) {
    const uint32_t p = RFq::mod_limb();
    const uint64_t G = __ballot(t < p);   // borrow generated
    const uint64_t E = __ballot(t == p);  // borrow propagated
    const uint64_t B = carries_in(G, E);
    const uint32_t bin = (uint32_t)(B >> __lane_id()) & 1u;
    const uint32_t d = t - p - bin;
    // final borrow out of limb 11 == borrow into lane 12 of this row: t < p -> keep t
    const bool lt = (B >> (rowdpp::row_shift() + 12)) & 1ull;
    return {lt ? t : d};
}

// resolve a redundant per-lane value (lo + carry-from-below <= 2^33 - 2) to canonical limbs
MBLS_DEV uint32_t rf_resolve(uint32_t lo, uint32_t carry_from_below) {
    const uint64_t s = (uint64_t)lo + carry_from_below;
    const uint32_t s_lo = (uint32_t)s;
    const uint64_t G = __ballot((s >> 32) != 0);
    const uint64_t P = __ballot(s_lo == 0xffffffffu);
    const uint64_t C = carries_in(G, P);
    return s_lo + ((uint32_t)(C >> __lane_id()) & 1u);
}

MBLS_DEV RFq operator+(const RFq& a, const RFq& b) {
    const uint64_t s = (uint64_t)a.v + b.v;  // <= 2^33 - 2
    const uint32_t t = rf_resolve((uint32_t)s, rowdpp::from_down((uint32_t)(s >> 32)));
    return rf_reduce_once(t);
}

MBLS_DEV RFq operator-(const RFq& a, const RFq& b) {
    const uint64_t G = __ballot(a.v < b.v);
    const uint64_t E = __ballot(a.v == b.v);
    const uint64_t B = carries_in(G, E);
    const bool limb = rowdpp::lane16() < 12;
    // padding lanes: the final borrow lands in lane 12 -- keep padding at zero
    const uint32_t d = limb ? a.v - b.v - ((uint32_t)(B >> __lane_id()) & 1u) : 0u;
    const bool neg = (B >> (rowdpp::row_shift() + 12)) & 1ull;
    if (!neg) return {d};
    // (a - b + 2^384) + p wraps past 2^384 exactly once: add lane-wise, drop the carry out
    const uint64_t s = (uint64_t)d + RFq::mod_limb();
    const uint32_t r = rf_resolve((uint32_t)s, rowdpp::from_down((uint32_t)(s >> 32)));
    return {limb ? r : 0u};
}

MBLS_DEV RFq neg(const RFq& a) { return RFq::zero() - a; }
MBLS_DEV RFq dbl(const RFq& a) { return a + a; }

// lane-parallel CIOS Montgomery product
MBLS_DEV RFq operator*(const RFq& a, const RFq& b) {
    const uint32_t p = RFq::mod_limb();
    uint64_t t = 0;  // redundant: value = sum_j t_j 2^(32 j), t_j < 2^34
#define MBLS_RF_ROW(I)                                                                    \
    {                                                                                     \
        const uint32_t bi = rowdpp::bcast<I>(b.v);                                        \
        const uint64_t v = (uint64_t)a.v * bi + t;                                        \
        const uint32_t m = rowdpp::bcast<0>((uint32_t)v) * FqCfg::NINV;                   \
        const uint64_t w = (uint64_t)m * p + (uint32_t)v;                                 \
        const uint64_t H = (uint64_t)(uint32_t)(v >> 32) + (uint32_t)(w >> 32);           \
        t = H + rowdpp::from_up((uint32_t)w);                                             \
    }
    MBLS_RF_ROW(0) MBLS_RF_ROW(1) MBLS_RF_ROW(2) MBLS_RF_ROW(3) MBLS_RF_ROW(4) MBLS_RF_ROW(5)
    MBLS_RF_ROW(6) MBLS_RF_ROW(7) MBLS_RF_ROW(8) MBLS_RF_ROW(9) MBLS_RF_ROW(10) MBLS_RF_ROW(11)
#undef MBLS_RF_ROW
    // t_j < 2^34: one ripple of the high parts, then carry-lookahead on the rest
    const uint32_t hi = (uint32_t)(t >> 32);  // <= 3
    const uint32_t r = rf_resolve((uint32_t)t, rowdpp::from_down(hi));
    return rf_reduce_once(r);
}

MBLS_DEV RFq sqr(const RFq& a) { return a * a; }

MBLS_DEV RFq inv(const RFq& a) {
    // Fermat a^(p-2), exponent bits are compile-time words (uniform control flow)
    RFq acc = RFq::one();
    for (int w = 11; w >= 0; --w) {
        const uint32_t e = FqCfg::MOD[w] - (w == 0 ? 2u : 0u);
        for (int bit = 31; bit >= 0; --bit) {
            acc = sqr(acc);
            if ((e >> bit) & 1u) acc = acc * a;
        }
    }
    return acc;
}

MBLS_DEV RFq from_mont(const RFq& a) {
    RFq one1 = {rowdpp::lane16() == 0 ? 1u : 0u};
    return a * one1;
}

// Fq2 over rows
struct RFq2 {
    RFq c0, c1;
    MBLS_DEV static RFq2 zero() { return {RFq::zero(), RFq::zero()}; }
    MBLS_DEV static RFq2 one() { return {RFq::one(), RFq::zero()}; }
    MBLS_DEV bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
    MBLS_DEV bool operator==(const RFq2& o) const { return c0 == o.c0 && c1 == o.c1; }
};
MBLS_DEV RFq2 operator+(const RFq2& a, const RFq2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
MBLS_DEV RFq2 operator-(const RFq2& a, const RFq2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
MBLS_DEV RFq2 neg(const RFq2& a) { return {neg(a.c0), neg(a.c1)}; }
MBLS_DEV RFq2 dbl(const RFq2& a) { return {dbl(a.c0), dbl(a.c1)}; }
MBLS_DEV RFq2 operator*(const RFq2& a, const RFq2& b) {
    RFq t0 = a.c0 * b.c0;
    RFq t1 = a.c1 * b.c1;
    RFq t2 = (a.c0 + a.c1) * (b.c0 + b.c1);
    return {t0 - t1, (t2 - t0) - t1};
}
MBLS_DEV RFq2 sqr(const RFq2& a) {
    RFq t = a.c0 * a.c1;
    return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
MBLS_DEV RFq2 inv(const RFq2& a) {
    RFq n = inv(sqr(a.c0) + sqr(a.c1));
    return {a.c0 * n, neg(a.c1 * n)};
}

// ---- memory: element `idx` of an array of 48-byte Fq; each row loads one element ------
MBLS_DEV RFq rf_load(const uint8_t* base, size_t idx) {
    const uint32_t j = rowdpp::lane16();
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + idx * 48);
    return {j < 12 ? p[j] : 0u};
}
MBLS_DEV void rf_store(uint8_t* base, size_t idx, const RFq& a) {
    const uint32_t j = rowdpp::lane16();
    uint32_t* p = reinterpret_cast<uint32_t*>(base + idx * 48);
    if (j < 12) p[j] = a.v;
}

// row counterpart of a scalar field type: Fq -> RFq, Fq2 -> RFq2
template <class F>
struct RowOf;
template <>
struct RowOf<Fq> {
    using type = RFq;
    static constexpr int FQS = 1;  // Fq elements per field element
    MBLS_DEV static RFq ld(const uint8_t* b, size_t fq_idx) { return rf_load(b, fq_idx); }
    MBLS_DEV static void st(uint8_t* b, size_t fq_idx, const RFq& v) { rf_store(b, fq_idx, v); }
};
template <>
struct RowOf<Fq2> {
    using type = RFq2;
    static constexpr int FQS = 2;
    MBLS_DEV static RFq2 ld(const uint8_t* b, size_t fq_idx) { return {rf_load(b, fq_idx), rf_load(b, fq_idx + 1)}; }
    MBLS_DEV static void st(uint8_t* b, size_t fq_idx, const RFq2& v) {
        rf_store(b, fq_idx, v.c0);
        rf_store(b, fq_idx + 1, v.c1);
    }
};

}  // namespace mbls
