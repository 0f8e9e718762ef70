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
#include "mbls_curve.hpp"

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

// Single-instruction lane ops whose carry / borrow lives in an SGPR lane mask.  A single wave
// issuing a dependent chain pays ~6 cycles per instruction whatever the operation
// (tools/latbench.hip), so the row arithmetic below is written for instruction COUNT: the carry
// mask of v_add_co_u32 IS the generate ballot, and v_addc / v_subb / v_cndmask take the
// lookahead result or a row-uniform flag directly as an SGPR mask (no per-lane bit extraction).
namespace rowop {
MBLS_DEV uint32_t add_co(uint32_t a, uint32_t b, uint64_t& carry) {
    uint32_t r;
    asm("v_add_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(carry) : "v"(a), "v"(b));
    return r;
}
MBLS_DEV uint32_t sub_co(uint32_t a, uint32_t b, uint64_t& borrow) {
    uint32_t r;
    asm("v_sub_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(borrow) : "v"(a), "v"(b));
    return r;
}
MBLS_DEV uint32_t add_mask(uint32_t a, uint64_t cin) {  // a + bit(cin, lane)
    uint32_t r;
    uint64_t c;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(c) : "v"(a), "s"(cin));
    return r;
}
MBLS_DEV uint32_t sub_mask(uint32_t a, uint64_t bin) {  // a - bit(bin, lane)
    uint32_t r;
    uint64_t c;
    asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(c) : "v"(a), "s"(bin));
    return r;
}
MBLS_DEV uint32_t pick(uint64_t m, uint32_t if0, uint32_t if1) {  // bit(m, lane) ? if1 : if0
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if0), "v"(if1), "s"(m));
    return r;
}
// every lane of row r <- bit 16 r + 12 of B (the carry / borrow out of limb 11 of that row)
MBLS_DEV uint64_t row_top_flag(uint64_t B) {
    const uint64_t y = (B >> 12) & 0x0001000100010001ull;
    return (y << 16) - y;  // row 3: the 2^64 term wraps away, leaving bits 48..63
}
}  // namespace rowop

// canonical r = t - p if t >= p else t   (t < 2p, canonical 32-bit limbs, padding lanes 0)
MBLS_DEV RFq rf_reduce_once(uint32_t t) {
    // every row's top limb below p's: t < p, nothing to subtract (a wave-uniform branch; ~half
    // of the sums of two canonical values)
    if ((__ballot(t < RFq::mod_limb()) & 0x0800080008000800ull) == 0x0800080008000800ull) return {t};
    uint64_t G;
    const uint32_t d = rowop::sub_co(t, RFq::mod_limb(), G);  // G: borrow generated
    const uint64_t E = __ballot(d == 0);                      // t_j == p_j: borrow propagated
    const uint64_t B = carries_in(G, E);
    const uint32_t r = rowop::sub_mask(d, B);
    // borrow out of limb 11 (t < p): keep t.  Padding lanes: t = 0, and r = 0 when t >= p
    return {rowop::pick(rowop::row_top_flag(B), r, t)};
}

// resolve a redundant per-lane value (lo + carry-from-below <= 2^33 - 2) to canonical limbs
MBLS_DEV uint32_t rf_resolve(uint32_t lo, uint32_t carry_from_below) {
    uint64_t G;
    const uint32_t s = rowop::add_co(lo, carry_from_below, G);
    const uint64_t P = __ballot(s == 0xffffffffu);
    return rowop::add_mask(s, carries_in(G, P));
}

MBLS_DEV RFq operator+(const RFq& a, const RFq& b) {
    // a + b < 2p < 2^384: the limb carries ARE the generate mask, no shifted carry word
    uint64_t G;
    const uint32_t s = rowop::add_co(a.v, b.v, G);
    const uint64_t P = __ballot(s == 0xffffffffu);
    return rf_reduce_once(rowop::add_mask(s, carries_in(G, P)));
}

MBLS_DEV RFq operator-(const RFq& a, const RFq& b) {
    uint64_t G;
    const uint32_t d0 = rowop::sub_co(a.v, b.v, G);
    const uint64_t E = __ballot(d0 == 0);
    const uint64_t B = carries_in(G, E);
    const uint32_t d = rowop::sub_mask(d0, B);  // a - b mod 2^384 (padding lane 12: -1 if a < b)
    const uint64_t neg = rowop::row_top_flag(B);
    if (neg == 0) return {d};  // no row borrowed: skip the correction (a wave-uniform branch)
    // a < b: (a - b + 2^384) + p wraps past 2^384 exactly once, which also clears lane 12
    uint64_t G2;
    const uint32_t e0 = rowop::add_co(d, RFq::mod_limb(), G2);
    const uint64_t P2 = __ballot(e0 == 0xffffffffu);
    const uint32_t e = rowop::add_mask(e0, carries_in(G2, P2));
    return {rowop::pick(neg, d, e)};
}

MBLS_DEV RFq neg(const RFq& a) { return RFq::zero() - a; }
MBLS_DEV RFq dbl(const RFq& a) { return a + a; }

// Unreduced operands for row products (the row counterparts of mbls_field.hpp's add_in / x2_in /
// x4_in): the row CIOS product returns < 2p, and its own conditional subtraction makes it
// canonical, whenever a * b < p * 2^384 -- e.g. an operand up to 8p against a canonical one
// (p < 2^381).  A shift by k is one row DPP move plus one v_alignbit per lane (no carry
// lookahead, no conditional subtraction): valid for a < 2^(384 - k), which also keeps the
// padding lane 12 zero.  add_in keeps the lookahead but skips the conditional subtraction.
template <int K>
MBLS_DEV RFq rf_shl(const RFq& a) {
    return {__builtin_amdgcn_alignbit(a.v, rowdpp::from_down(a.v), 32 - K)};
}
MBLS_DEV RFq x2_in(const RFq& a) { return rf_shl<1>(a); }
MBLS_DEV RFq x4_in(const RFq& a) { return rf_shl<2>(a); }
MBLS_DEV RFq x8_in(const RFq& a) { return rf_shl<3>(a); }
MBLS_DEV RFq add_in(const RFq& a, const RFq& b) {  // a + b < 2^384, no reduction
    uint64_t G;
    const uint32_t s = rowop::add_co(a.v, b.v, G);
    const uint64_t P = __ballot(s == 0xffffffffu);
    return {rowop::add_mask(s, carries_in(G, P))};
}

// lane-parallel CIOS Montgomery product.  Round i, lane j:  v = a_j b_i + t_j,
// m = lo(v_0) (-p^-1), w = m p_j + lo(v_j), t_j <- hi(v_j) + hi(w_j) + lo(w_{j+1}).
// The round's dependent chain is what a lone wave pays for (tools/latbench.hip), so m is taken
// from t_0 directly:  lo(v_0) (-p^-1) = lo(t_0) (-p^-1) + (a_0 (-p^-1)) b_i  (mod 2^32), one
// v_mad_u64_u32 on the broadcast lo(t_0) with the addend a_0 (-p^-1) b_i computed off the chain,
// while v = a b_i + t runs beside it:  bcast -> mad (m) -> mad (w) -> row shift -> add per round
// instead of mad (v) -> bcast -> mul (m) -> mad (w) -> row shift -> add.
MBLS_DEV uint32_t rf_mad_lo(uint32_t x, uint32_t y, uint32_t z) {  // lo(x*y + z) in ONE instruction
    uint64_t r, c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(c) : "v"(x), "s"(y), "v"((uint64_t)z));
    return (uint32_t)r;
}
// 64-bit sum of two 32-bit values (opaque to the scheduler: keeps hi(v) + hi(w) off the row shift's
// critical path instead of being reassociated behind it)
MBLS_DEV uint64_t rf_add32x2(uint32_t x, uint32_t y) {
    uint32_t lo, hi;
    uint64_t c;
    asm("v_add_co_u32_e64 %0, %2, %3, %4\n\tv_addc_co_u32_e64 %1, %2, 0, 0, %2"
        : "=&v"(lo), "=v"(hi), "=&s"(c)
        : "v"(x), "v"(y));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// (hi:lo) + x as a register pair, x 32-bit
MBLS_DEV uint64_t rf_add64_32(uint64_t h, uint32_t x) {
    uint32_t lo, hi;
    uint64_t c;
    asm("v_add_co_u32_e64 %0, %2, %3, %4\n\tv_addc_co_u32_e64 %1, %2, %5, 0, %2"
        : "=&v"(lo), "=v"(hi), "=&s"(c)
        : "v"((uint32_t)h), "v"(x), "v"((uint32_t)(h >> 32)));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
MBLS_DEV RFq operator*(const RFq& a, const RFq& b) {
    const uint32_t p = RFq::mod_limb();
    const uint32_t ninv = __builtin_amdgcn_readfirstlane(FqCfg::NINV);
    const uint32_t a0n = rowdpp::bcast<0>(a.v) * FqCfg::NINV;
    uint64_t t = 0;  // redundant: value = sum_j t_j 2^(32 j), t_j < 2^34
#define MBLS_RF_ROW(I)                                                                    \
    {                                                                                     \
        const uint32_t bi = rowdpp::bcast<I>(b.v);                                        \
        const uint32_t m = rf_mad_lo(rowdpp::bcast<0>((uint32_t)t), ninv, a0n * bi);      \
        const uint64_t v = (uint64_t)a.v * bi + t;                                        \
        const uint64_t w = (uint64_t)m * p + (uint32_t)v;                                 \
        const uint64_t H = rf_add32x2((uint32_t)(v >> 32), (uint32_t)(w >> 32));          \
        t = rf_add64_32(H, rowdpp::from_up((uint32_t)w));                                 \
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

// a row-sliced square is a full row product: the curve formulas use products instead of
// squares-plus-additions (mbls_curve.hpp SqrCheaper)
template <>
struct SqrCheaper<RFq> {
    static constexpr bool value = false;
};
template <>
struct SqrCheaper<RFq2> {
    static constexpr bool value = false;
};
template <>
struct ShiftOperands<RFq> {
    static constexpr bool value = true;
};

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
