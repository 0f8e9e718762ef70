// mbls_fq2_28.hpp -- pair-sliced Fq2 in unsaturated radix 2^28 for the G2 accumulation (round 6).
//
// The G2 lane kernels hold one Fq2 element c0 + c1 u in a PAIR of adjacent lanes (lane 2k: c0,
// lane 2k+1: c1; mbls_pairfield.hpp) and turn every Fq2 product into ONE Fq product sum per lane.
// Here the lane's component is a radix-2^28 r28::F28 (mbls_fq28.hpp): a column is one
// v_mad_u64_u32 chain with no carry tracking, so a lane's product sum costs ~660 instead of ~940
// instructions (the FIPS fips::mul2 pays a v_addc per mad; tools/isa counts in DESIGN.md):
//     mul:  lane 0  a0 b0 + a1 (K p - b1)       lane 1  a1 b0 + a0 b1          (r28::mul2)
//     sqr:  lane 0  (a0 + a1)(a0 - a1 + K p)    lane 1  a1 (2 a0)              (r28::mul)
//     mul2: the two products' terms, one reduction                             (r28::mul4)
// The partner's limbs arrive by one DPP quad_perm move per limb.  Additions, biased subtractions,
// carries and folds are per component.
//
// Bounds.  Every step of madd / mmadd below is restated limb for limb in tests/limbs_model.py
// (_fq2_formulas), which asserts each column stays below 2^64 on the extreme operands of
// tests/test_gpu_limbs.py (accumulators at their invariant bounds, bases at the unpack extremes,
// negated y carried): the largest column seen is 2^62.44.  The rules that keep it there:
//   * product operands are normalised (limbs < 2^28), except the partner negations K p - b (limbs
//     < 2^30.4) and the squares' a0 +- a1 -- so H, R2, V - X3 and -2 Y1 are carried first;
//   * a partner negation takes the smallest bias whose limbs, the top one included, cover the
//     operand: B16 for values < 16 p, B32 < 32 p, B512 beyond (x4(HH), R2);
//   * the invariant between steps: x, y folded (normalised, < 3p), z normalised.
// Same field values as jac_madd / jac_mmadd over PFq2 (madd-2007-bl, lazy Y3, Z3 = 2 Z1 H), hence
// the same Jacobian partials bit for bit after the final conversion to words.
#pragma once
#include "mbls_curve.hpp"
#include "mbls_fq28.hpp"
#include "mbls_pairfield.hpp"

namespace mbls {
namespace r28p {

using r28::F28;

MBLS_DEV F28 partner(const F28& a) {
    F28 r;
#pragma unroll
    for (int i = 0; i < r28::NL; ++i) r.l[i] = pairdpp::swap(a.l[i]);
    return r;
}
MBLS_DEV F28 sel(bool c, const F28& a, const F28& b) {
    F28 r;
#pragma unroll
    for (int i = 0; i < r28::NL; ++i) r.l[i] = c ? a.l[i] : b.l[i];
    return r;
}
// a predicate of this lane's component, true when it holds on both lanes of the pair
MBLS_DEV bool both(bool p) {
    const uint32_t v = p ? 1u : 0u;
    return (v & pairdpp::swap(v)) != 0;
}

// this lane's component of the Fq2 product a b (BK: bias of the partner's negated b1)
template <const uint32_t* BK>
MBLS_DEV F28 mul(const F28& a, const F28& b) {
    const bool j = pairdpp::odd();
    const F28 y = partner(a), bp = partner(b);
    return r28::mul2(a, sel(j, bp, b), y, sel(j, b, r28::neg<BK>(bp)));
}
// a^2 (BK: bias of a0 - a1)
template <const uint32_t* BK>
MBLS_DEV F28 sqr(const F28& a) {
    const bool j = pairdpp::odd();
    const F28 y = partner(a);
    return r28::mul(sel(j, a, r28::add(a, y)), sel(j, r28::x2(y), r28::sub<BK>(a, y)));
}
// a b + c d with one reduction per lane
template <const uint32_t* BKB, const uint32_t* BKD>
MBLS_DEV F28 mul2(const F28& a, const F28& b, const F28& c, const F28& d) {
    const bool j = pairdpp::odd();
    const F28 ya = partner(a), bp = partner(b), yc = partner(c), dp = partner(d);
    return r28::mul4(a, sel(j, bp, b), ya, sel(j, b, r28::neg<BKB>(bp)), c, sel(j, dp, d), yc,
                     sel(j, d, r28::neg<BKD>(dp)));
}
// the Fq2 value is 0 mod p (components normalised, < 2p)
MBLS_DEV bool is_zero_lt2p(const F28& a) { return both(r28::is_zero_lt2p(a)); }

// R'-one of Fq2 on this lane: (ONE, 0)
MBLS_DEV F28 one() { return pairdpp::odd() ? F28::zero() : F28::one(); }

// Jacobian accumulator (this lane's components); infinity is exactly z = 0 on both lanes
struct J28p {
    F28 x, y, z;
    MBLS_DEV bool is_inf() const {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < r28::NL; ++i) t |= z.l[i];
        return both(t == 0);
    }
    MBLS_DEV static J28p inf() { return {one(), one(), F28::zero()}; }
};

// acc + q (q = (x2, y2) from unpack_shift8, y2 carried after a negation; not the identity).
// Returns false, acc untouched, when H = 0 (equal or opposite points): the caller takes the
// word-form path (jac_madd over PFq2) for that rare step.
MBLS_DEV bool madd(J28p& acc, const F28& x2_, const F28& y2_) {
    using namespace r28;
    const F28 Z1Z1 = r28p::sqr<B16>(acc.z);
    const F28 H = carry(sub<B16>(r28p::mul<B16>(x2_, Z1Z1), acc.x));  // < 19p
    const F28 HH = r28p::sqr<B32>(H);
    if (r28p::is_zero_lt2p(HH)) return false;
    const F28 R = sub<B16>(r28p::mul<B16>(r28p::mul<B16>(y2_, acc.z), Z1Z1), acc.y);
    const F28 I = x4(HH);
    const F28 J = r28p::mul<B512>(H, I);
    acc.z = r28p::mul<B32>(x2(acc.z), H);
    const F28 V = r28p::mul<B512>(acc.x, I);
    const F28 R2 = carry(x2(R));  // < 38p
    acc.x = fold(sub<B32>(sub<B16>(r28p::sqr<B512>(R2), J), x2(V)));
    acc.y = r28p::mul2<B32, B16>(R2, carry(sub<B16>(V, acc.x)), carry(neg<B32>(x2(acc.y))), J);
    return true;
}

// acc fresh from the chunk's first point (z = R'-one, x, y folded): mmadd-2007-bl, Z3 = 2H.
// Returns false (acc untouched) when x1 == x2 mod p, left to madd's branches.
MBLS_DEV bool mmadd(J28p& acc, const F28& x2_, const F28& y2_) {
    using namespace r28;
    const F28 H = fold(sub<B512>(x2_, acc.x));
    const F28 HH = r28p::sqr<B16>(H);
    if (r28p::is_zero_lt2p(HH)) return false;
    const F28 I = x4(HH);
    const F28 J = r28p::mul<B512>(H, I);
    const F28 V = r28p::mul<B512>(acc.x, I);
    const F28 R2 = carry(x2(fold(sub<B512>(y2_, acc.y))));
    acc.z = carry(x2(H));
    acc.x = fold(sub<B32>(sub<B16>(r28p::sqr<B16>(R2), J), x2(V)));
    acc.y = r28p::mul2<B32, B16>(R2, carry(sub<B16>(V, acc.x)), carry(neg<B32>(x2(acc.y))), J);
    return true;
}

// ------------------------------------------------------------------------- XYZZ (round 6)
// The G1 accumulation's XYZZ forms (mbls_fq28.hpp: madd-2008-s, add-2008-s, dbl-2008-s-1) over
// pair-sliced Fq2: one squaring fewer per mixed addition (an r28 product per lane), two per full
// addition.  Every product operand is carried first and every partner negation takes the bias
// rule above; tests/limbs_model.py (_fq2_xyzz_formulas) restates each step and checks the columns.
// Invariant between steps: x, y folded (normalised, < 3p); zz, zzz normalised, < 3p.
struct X28p {
    F28 x, y, zz, zzz;
    MBLS_DEV bool is_inf() const {
        uint32_t t = 0;
#pragma unroll
        for (int i = 0; i < r28::NL; ++i) t |= zz.l[i];
        return both(t == 0);
    }
    MBLS_DEV static X28p inf() { return {one(), one(), F28::zero(), F28::zero()}; }
};
// the Fq2 value is 0 mod p (any components < 2^391)
MBLS_DEV bool is_zero_mod(const F28& a) { return both(r28::is_zero_mod(a)); }

MBLS_DEV void xdbl(X28p& a) {
    using namespace r28;
    const F28 U = carry(x2(a.y));  // < 6p
    const F28 V = r28p::sqr<B16>(U);
    const F28 W = r28p::mul<B16>(U, V);
    const F28 S = r28p::mul<B16>(a.x, V);
    const F28 A = r28p::sqr<B16>(a.x);
    const F28 M = carry(add(x2(A), A));  // 3 X^2, < 6p
    const F28 X3 = fold(sub<B32>(r28p::sqr<B16>(M), x2(S)));
    a.y = r28p::mul2<B32, B16>(M, carry(sub<B16>(S, X3)), carry(neg<B16>(a.y)), W);
    a.x = X3;
    a.zz = r28p::mul<B16>(V, a.zz);
    a.zzz = r28p::mul<B16>(W, a.zzz);
}

// acc + q (q = (x2, y2) from unpack_shift8, y2 carried after a negation; not the identity)
MBLS_DEV void xmadd(X28p& acc, const F28& x2_, const F28& y2_) {
    using namespace r28;
    if (acc.is_inf()) {
        acc = {fold(x2_), fold(y2_), one(), one()};
        return;
    }
    const F28 U2 = r28p::mul<B16>(x2_, acc.zz);
    const F28 S2 = r28p::mul<B16>(y2_, acc.zzz);
    const F28 Pd = carry(sub<B16>(U2, acc.x));  // < 18p
    const F28 R = carry(sub<B16>(S2, acc.y));   // < 18p
    const F28 PP = r28p::sqr<B32>(Pd);
    if (r28p::is_zero_lt2p(PP)) {  // equal or opposite points
        if (r28p::is_zero_mod(R))
            xdbl(acc);
        else
            acc = X28p::inf();
        return;
    }
    acc.zz = r28p::mul<B16>(acc.zz, PP);
    const F28 PPP = r28p::mul<B16>(Pd, PP);
    acc.zzz = r28p::mul<B16>(acc.zzz, PPP);
    const F28 Q = r28p::mul<B16>(acc.x, PP);
    acc.x = fold(sub<B32>(sub<B16>(r28p::sqr<B32>(R), PPP), x2(Q)));
    acc.y = r28p::mul2<B32, B16>(R, carry(sub<B16>(Q, acc.x)), carry(neg<B16>(acc.y)), PPP);
}

// acc fresh from the chunk's first point (zz = zzz = one, x, y folded) + q: ZZ = PP, ZZZ = PPP.
// Returns false (acc untouched) when x1 == x2 mod p, left to xmadd's branches.
MBLS_DEV bool xmmadd(X28p& acc, const F28& x2_, const F28& y2_) {
    using namespace r28;
    const F28 Pd = fold(sub<B512>(x2_, acc.x));
    const F28 PP = r28p::sqr<B16>(Pd);
    if (r28p::is_zero_lt2p(PP)) return false;
    const F28 R = fold(sub<B512>(y2_, acc.y));
    const F28 PPP = r28p::mul<B16>(Pd, PP);
    const F28 Q = r28p::mul<B16>(acc.x, PP);
    const F28 X3 = fold(sub<B32>(sub<B16>(r28p::sqr<B16>(R), PPP), x2(Q)));
    acc.y = r28p::mul2<B32, B16>(R, carry(sub<B16>(Q, X3)), carry(neg<B16>(acc.y)), PPP);
    acc.x = X3;
    acc.zz = PP;
    acc.zzz = PPP;
    return true;
}

// acc + a partial (x2, y2, zz2, zzz2): a stored accumulator's raw limbs (normalised, < 3p), zz2 != 0
MBLS_DEV void xadd(X28p& acc, const F28& x2_, const F28& y2_, const F28& zz2, const F28& zzz2) {
    using namespace r28;
    if (acc.is_inf()) {
        acc = {x2_, y2_, zz2, zzz2};
        return;
    }
    const F28 U1 = r28p::mul<B16>(acc.x, zz2);
    const F28 U2 = r28p::mul<B16>(x2_, acc.zz);
    const F28 S1 = r28p::mul<B16>(acc.y, zzz2);
    const F28 S2 = r28p::mul<B16>(y2_, acc.zzz);
    const F28 Pd = carry(sub<B16>(U2, U1));
    const F28 R = carry(sub<B16>(S2, S1));
    const F28 PP = r28p::sqr<B32>(Pd);
    if (r28p::is_zero_lt2p(PP)) {
        if (r28p::is_zero_mod(R))
            xdbl(acc);
        else
            acc = X28p::inf();
        return;
    }
    const F28 PPP = r28p::mul<B16>(Pd, PP);
    const F28 Q = r28p::mul<B16>(U1, PP);
    acc.zz = r28p::mul<B16>(r28p::mul<B16>(acc.zz, zz2), PP);
    acc.zzz = r28p::mul<B16>(r28p::mul<B16>(acc.zzz, zzz2), PPP);
    acc.x = fold(sub<B32>(sub<B16>(r28p::sqr<B32>(R), PPP), x2(Q)));
    acc.y = r28p::mul2<B32, B16>(R, carry(sub<B16>(Q, acc.x)), carry(neg<B16>(S1)), PPP);
}

// XYZZ -> Jacobian (X ZZ^2, Y ZZZ^2, ZZZ)
MBLS_DEV J28p x_to_jac(const X28p& a) {
    using r28::B16;
    if (a.is_inf()) return J28p::inf();
    return {r28p::mul<B16>(a.x, r28p::sqr<B16>(a.zz)), r28p::mul<B16>(a.y, r28p::sqr<B16>(a.zzz)), a.zzz};
}

// this lane's component to / from the library's canonical Montgomery words (x R mod p)
MBLS_DEV PFq2 to_pf(const F28& a) {
    PFq2 r;
    r28::to_words(a, r.v.v);
    return r;
}
MBLS_DEV F28 from_pf(const PFq2& a) { return r28::unpack_shift8(a.v.v); }

}  // namespace r28p
}  // namespace mbls
