// mbls_pairfield.hpp -- "pair-sliced" Fq2 arithmetic for the throughput-bound G2 kernels.
//
// One Fq2 element c0 + c1 u lives in a PAIR of adjacent lanes: lane 2k holds c0, lane 2k+1
// holds c1 (12 x u32 limbs each).  Every Fq2 product is then exactly one lazy-reduced Fq
// product-sum per lane (fips::mul2):
//     lane 0: c0 = a0*b0 + a1*(-b1)        lane 1: c1 = a1*b0 + a0*b1
// and a square one Fq product per lane:
//     lane 0: c0 = (a0 + a1)(a0 - a1)      lane 1: c1 = 2 a0 a1
// The partner's limbs arrive through one DPP quad_perm move per limb.  Total VALU work equals
// the scalar Karatsuba form (3 x 288 vs 2 x 432 mads) but each lane holds Fq-sized values, so
// the G2 accumulation runs at the register footprint of G1 (no spills, >1 wave per SIMD)
// instead of 256 VGPRs + 136 AGPRs + 1 KB of scratch per lane for the scalar Fq2 kernel.
//
// Requirement: both lanes of a pair are active together (pairs diverge only as a whole);
// every predicate below (is_zero, ==) is combined over the pair, so control flow that depends
// on field values stays pair-uniform.  Storage layout is unchanged (Fq2 = c0 || c1, 96 B):
// lane j loads / stores the 48 bytes of component j.
#pragma once
#include "mbls_field.hpp"

namespace mbls {

namespace pairdpp {
// quad_perm [1,0,3,2]: lane i <- lane i^1
MBLS_DEV uint32_t swap(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, false); }
MBLS_DEV bool odd() { return (__lane_id() & 1) != 0; }
}  // namespace pairdpp

MBLS_DEV Fq partner(const Fq& a) {
    Fq r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r.v[i] = pairdpp::swap(a.v[i]);
    return r;
}
MBLS_DEV Fq select(bool c, const Fq& a, const Fq& b) {
    Fq r;
#pragma unroll
    for (int i = 0; i < 12; ++i) r.v[i] = c ? a.v[i] : b.v[i];
    return r;
}

struct PFq2 {
    Fq v;  // this lane's component: c0 on even lanes, c1 on odd lanes

    MBLS_DEV static PFq2 zero() { return {Fq::zero()}; }
    MBLS_DEV static PFq2 one() { return {select(pairdpp::odd(), Fq::zero(), Fq::one())}; }
    MBLS_DEV bool is_zero() const {
        const uint32_t z = v.is_zero() ? 1u : 0u;
        return (z & pairdpp::swap(z)) != 0;
    }
    MBLS_DEV bool operator==(const PFq2& o) const {
        const uint32_t e = (v == o.v) ? 1u : 0u;
        return (e & pairdpp::swap(e)) != 0;
    }
};

MBLS_DEV PFq2 operator+(const PFq2& a, const PFq2& b) { return {a.v + b.v}; }
MBLS_DEV PFq2 operator-(const PFq2& a, const PFq2& b) { return {a.v - b.v}; }
MBLS_DEV PFq2 neg(const PFq2& a) { return {neg(a.v)}; }
MBLS_DEV PFq2 dbl(const PFq2& a) { return {dbl(a.v)}; }

MBLS_DEV PFq2 operator*(const PFq2& a, const PFq2& b) {
    const bool j = pairdpp::odd();
    const Fq y = partner(a.v);   // a_(1-j)
    const Fq bp = partner(b.v);  // b_(1-j)
    // lane 0: a0*b0 + a1*(-b1); lane 1: a1*b0 + a0*b1 (-b1 as p - b1, unreduced: the lazy sum stays
    // below 2p^2)
    return {fips::mul2(a.v, select(j, bp, b.v), y, select(j, b.v, neg_in(bp)))};
}

MBLS_DEV PFq2 sqr(const PFq2& a) {
    const bool j = pairdpp::odd();
    const Fq y = partner(a.v);
    // lane 0: (a0 + a1)(a0 - a1); lane 1: a1 (2 a0).  a0 + a1 and 2 a0 feed only the product:
    // unreduced (< 2p against a canonical partner, mbls_field.hpp add_in), and the product's own
    // conditional subtraction leaves both lanes canonical
    return {select(j, a.v, add_in(a.v, y)) * select(j, x2_in(y), a.v - y)};
}

MBLS_DEV PFq2 inv(const PFq2& a) {
    const Fq y = partner(a.v);
    const Fq n = inv(sqr(a.v) + sqr(y));  // a0^2 + a1^2 on both lanes
    const Fq r = a.v * n;
    return {select(pairdpp::odd(), neg(r), r)};
}

}  // namespace mbls
